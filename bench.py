"""ResNet-18 TQ (g=8, alpha=k=12, wb=db=9, dt=3) inference throughput on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 256]
        (N > 1 without a launcher: bench.py starts N fresh rank processes itself, before any
        GPU call, rendezvous on 127.0.0.1)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one TQ forward of one synthetic 256x3x224x224 batch per GPU (BASELINE.json
configs[1]) through the fused executor (tq_fuse.py): the stem (conv, BN,
ReLU, max-pool, first codes) is one HIP kernel, the 19 converted convs run the term-pair
kernels with BN/residual/ReLU/next-layer TR in their epilogue; avgpool and fc are torch on
the same stream.  By default each batch is split into two 128-image chunks on two HIP
streams, launched layer by layer round-robin and replayed as one captured hipGraph, so one
chunk's kernels fill the CUs the other's leave idle while they drain (bit-identical logits;
--streams 1 --launch eager is the plain one-stream loop).  The kernel rooflines come from a
separate one-stream pass with full-batch launches.  Inputs are resident in HBM before timing.  Ranks run independent batches (weak
scaling, no data-path collective); one all-reduce of the accuracy counters closes the
timed region.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))

import cnn_models  # noqa: E402
import profile_model  # noqa: E402
import tq_fuse  # noqa: E402
import tq_ops  # noqa: E402
import tr_layer  # noqa: E402
import util  # noqa: E402

METRIC = "term-pair MACs/sec + images/sec, ResNet-18 TQ g=8 at 1/2/4/8 MI355X"
WB, G, K, DB, DT = 9, 8, 12, 9, 3
STEM_NAMES = {"fused": "split-fp16 near-fp32 (fused stem kernel; its codes sit closer to the "
                       "correctly rounded conv's than torch's fp32 convs do, DESIGN 3)",
              "exact": "correctly rounded codes (fused stem kernel + exact fp64 recompute of "
                       "every output within the split's error bound of a rounding midpoint)",
              "fp32": "torch fp32 conv (MIOpen) + BN/ReLU/max-pool/codes kernel"}
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md chip table (spec)
HBM_BYTES_PER_IMAGE = 15026432   # algorithmic bytes of the TR path per image
VALU_LANE_OPS = 256 * 4 * 32 * 2.4e9   # CUs x SIMDs x lanes x clock = 78.6e12 lane-op/s
# v_dot2c_i32_i16 issues at half the VALU rate on gfx950 (4 cycles per wave64; measured
# 35.8e12 lane-op/s by tools/valu_peak.hip) and does 2 int16 MACs per lane-op:
DOT2_PEAK = 2 * VALU_LANE_OPS / 2   # 78.6e12 term-sum MAC/s
# v_mfma_f32_32x32x16_f16: dense fp16 MFMA peak (MI355X_MICROARCH.md, matrix cores; the
# 2:1-sparsity headline is not a dense rate) -- 2 FLOP per term-sum product
MFMA_F16_PEAK_TFLOPS = 2500.0
FP32_PEAK_TFLOPS = 157.3         # MI355X fp32 vector / f32-MFMA peak (MI355X_MICROARCH.md)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--cpu-sample", type=int, default=256,
                    help="images in the CPU-baseline sample (rank 0, N=1 only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--engine", choices=("mfma", "valu"), default="mfma",
                    help="term-pair engine: MFMA (fp16 codes) or VALU (int16 codes, "
                         "v_dot2c_i32_i16); bit-identical outputs")
    ap.add_argument("--launch", choices=("graph", "eager"), default="graph",
                    help="graph: replay each resident batch's forward as a captured hipGraph "
                         "(no per-kernel host launches: +1.7 %% at 2 streams, equal at 1); "
                         "eager: launch from Python every step")
    ap.add_argument("--graph", action="store_true", help="same as --launch graph")
    ap.add_argument("--streams", type=int, default=2,
                    help="fused executor: split each batch into this many image chunks, one "
                         "HIP stream each, launches issued layer by layer round-robin (2: "
                         "each kernel's drain overlaps the other chunk's kernel; 1 = one "
                         "stream)")
    ap.add_argument("--no-d1", action="store_true",
                    help="skip the d1_tr_op key (SURVEY 8(d) D1: the TR op alone)")
    ap.add_argument("--no-d4", action="store_true",
                    help="skip the d4 key (BASELINE configs[2]/[3]: LSTM-650, fused "
                         "MobileNet-V2 / EfficientNet-b0; rank 0 at N=1 only)")
    ap.add_argument("--stem", choices=("fused", "exact", "fp32"), default="exact",
                    help="exact: the fused stem kernel (split-fp16 MFMA conv) + its exact "
                         "fix-up (the codes of the correctly rounded fp32 conv); fused: the "
                         "fused stem kernel alone (near-fp32); fp32: torch's fp32 conv + the "
                         "BN/ReLU/max-pool/codes kernel")
    ap.add_argument("--no-stem-leg", action="store_true",
                    help="skip the second timed pass with the other stem (N=1 only)")
    ap.add_argument("--unfused", action="store_true",
                    help="run the module path (separate BN/ReLU/add/TR passes) instead of "
                         "the fused executor")
    ap.add_argument("--dry-launch", action="store_true",
                    help="launcher check only (tests): each rank prints its rank and world "
                         "size as JSON and exits before touching the GPU")
    return ap.parse_args(argv)


def launch_plan(gpus, env):
    """What this process does for ``--gpus N`` given the environment: ("spawn", N) when no
    launcher set WORLD_SIZE and N > 1 (this process starts N fresh rank processes before any
    GPU call), ("run", world) when WORLD_SIZE agrees with N (or N = 1 without a launcher),
    else ("error", message): a mismatch never silently measures another GPU count."""
    if gpus < 1:
        return ("error", "--gpus must be >= 1")
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return ("spawn", gpus) if gpus > 1 else ("run", 1)
    if int(ws) != gpus:
        return ("error", "--gpus %d but WORLD_SIZE=%s: launch with --nproc-per-node %d, or "
                         "without a launcher to let bench.py start the ranks" % (gpus, ws, gpus))
    return ("run", gpus)


def spawn_ranks(argv, n, dry, timeout_s=None, poll_s=0.2):
    """Start ranks 0..n-1 as fresh processes, one per GPU, rendezvous on 127.0.0.1; return
    non-zero if any rank fails.  This process never touches torch.cuda (not even
    device_count(), which falls back to hipGetDeviceCount when amdsmi fails and would then
    initialise HIP in the parent of every rank): each rank checks the visible GPU count
    itself (check_world).  The children are polled: when one exits non-zero the others are
    terminated (a rank stuck in init or a collective would otherwise block until the process
    group times out), and all of them when the overall time limit (TQ_BENCH_SPAWN_TIMEOUT
    seconds, default 3600) passes."""
    import socket
    import subprocess
    import time
    if timeout_s is None:
        timeout_s = float(os.environ.get("TQ_BENCH_SPAWN_TIMEOUT", "3600"))
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env))
    t_end = time.monotonic() + timeout_s
    failed = False
    while True:
        rcs = [p.poll() for p in procs]
        if any(rc not in (None, 0) for rc in rcs):
            failed = True
            print("bench.py: a rank exited with %s; stopping the others" %
                  [rc for rc in rcs if rc not in (None, 0)][0], file=sys.stderr)
            break
        if all(rc == 0 for rc in rcs):
            return 0
        if time.monotonic() > t_end:
            failed = True
            print("bench.py: ranks still running after %.0f s; stopping them" % timeout_s,
                  file=sys.stderr)
            break
        time.sleep(poll_s)
    for p in procs:
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return 1 if failed else 0


def check_world(world, local):
    """A rank's own check that its GPU exists (spawn_ranks leaves the count to the ranks).
    Per node: the ranks of this node (LOCAL_WORLD_SIZE, torchrun's; WORLD_SIZE when unset)
    must fit its visible GPUs, so a multi-node torchrun (WORLD_SIZE > GPUs per node) passes."""
    have = torch.cuda.device_count()
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    if local >= have or local_world > have:
        print("bench.py: %d rank(s) on this node (local rank %d, world size %d) but only %d "
              "GPU(s) visible" % (local_world, local, world, have), file=sys.stderr)
        return False
    return True


class KernelTimer(object):
    """HIP events around the TQ kernels inside the timed region (tq_ops hook)."""

    def __init__(self):
        self.events = {}
        self.work = {}
        self.nbytes = {}
        self.per_launch = {}  # name -> [(work, bytes)] in launch order
        # time base on the launching stream: every kernel event (on any chunk stream, each
        # of which first waits on this stream) comes after it on the device timeline
        self.base = torch.cuda.Event(enable_timing=True)
        self.base.record(torch.cuda.current_stream())

    def __call__(self, name, work, fn, nbytes=0):
        s = torch.cuda.current_stream()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(s)
        r = fn()
        b.record(s)
        self.events.setdefault(name, []).append((a, b))
        self.per_launch.setdefault(name, []).append((work, nbytes))
        self.work[name] = self.work.get(name, 0) + work
        self.nbytes[name] = self.nbytes.get(name, 0) + nbytes
        return r

    def summary(self):
        """Per kernel name: launches, summed launch durations ("seconds") and the time at
        least one launch of it is running ("busy": the union of the launch intervals, which
        equals "seconds" on one stream and is shorter when chunk streams overlap them)."""
        out = {}
        for name, evs in self.events.items():
            iv = sorted((self.base.elapsed_time(a), self.base.elapsed_time(b)) for a, b in evs)
            t = sum(e - s for s, e in iv) * 1e-3
            busy, cur_s, cur_e = 0.0, None, None
            for s, e in iv:
                if cur_e is None or s > cur_e:
                    if cur_e is not None:
                        busy += cur_e - cur_s
                    cur_s, cur_e = s, e
                else:
                    cur_e = max(cur_e, e)
            if cur_e is not None:
                busy += cur_e - cur_s
            out[name] = {"launches": len(evs), "seconds": t, "busy": busy * 1e-3,
                         "work": self.work[name], "bytes": self.nbytes[name],
                         "per_launch": self.per_launch[name]}
        return out


def build_model(dev, batch, seed):
    torch.manual_seed(0)
    model = cnn_models.resnet18(pretrained=False).to(dev).eval()
    settings = cnn_models.static_conv_layer_settings(model, WB, G, K)
    qmodel = cnn_models.convert_model(model, settings, DB, DT)
    qmodel = qmodel.to(memory_format=torch.channels_last)
    assert all(m.termpair for m in qmodel.modules() if isinstance(m, tr_layer.TRConv2dLayer))
    engines = {m.engine for m in qmodel.modules() if isinstance(m, tr_layer.TRConv2dLayer)}
    assert engines == {os.environ["TQ_CONV_ENGINE"]}, engines
    # term-pair MACs per image (profile_model, 1x3x224x224 -- evaluate_cnn.py:28-29)
    tmacs, _ = profile_model.get_model_ops(qmodel, (torch.randn(1, 3, 224, 224, device=dev),))
    # calibration: one tracking pass on this rank's calibration batch, histograms summed
    # over ranks, then every rank runs the same mse_profile
    calib = util.SyntheticImageNet(batch, batch, seed=1000 + seed, device=dev).batch(0)[0]
    with torch.no_grad():
        qmodel(calib.to(memory_format=torch.channels_last))
    util.allreduce_histograms(qmodel)
    tr_layer.set_tr_tracking(qmodel, False)
    return model, qmodel, tmacs


def host_info():
    """CPU of this host: model name (/proc/cpuinfo), logical CPUs (nproc) and the threads a
    baseline may use (OMP_NUM_THREADS: 16 on the GPU box, its CPU share; else nproc)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    threads = int(os.environ.get("OMP_NUM_THREADS") or nproc)
    return model, nproc, max(1, min(threads, nproc))


def cpu_baseline(model_fp, qmodel, nimg):
    """The reference algorithm on the host, on all the CPU threads this job may use: the
    oracle (C restatement of the reference kernel) TR-ing every TR-layer activation, split in
    chunks over a thread pool (g = 1 is elementwise; ctypes releases the GIL), and the
    reference's dense fp32 torch conv (torch.set_num_threads) on the fake-quantized tensors;
    timed on a bounded sample of the bench workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    import copy
    import torch.nn as nn
    from concurrent.futures import ThreadPoolExecutor
    cpu_model, nproc, threads = host_info()
    pool = ThreadPoolExecutor(threads)

    def tr_parallel(x, sf, db, dt):
        flat = x.contiguous().numpy().reshape(-1)
        out = np.empty_like(flat)
        bounds = np.linspace(0, flat.size, 4 * threads + 1).astype(np.int64)

        def run(j):
            lo, hi = bounds[j], bounds[j + 1]
            if hi > lo:
                out[lo:hi] = oracle.tr(flat[lo:hi].reshape(1, -1, 1, 1), sf, db, 1,
                                       dt).reshape(-1)
        list(pool.map(run, range(4 * threads)))
        return torch.from_numpy(out).view(x.shape)

    class OracleTRConv(nn.Module):
        def __init__(self, layer):
            super(OracleTRConv, self).__init__()
            self.conv = copy.deepcopy(layer.conv).cpu().float()
            self.sf = layer.input_quant.sf
            self.db, self.dt = layer.data_bits, layer.data_terms

        def forward(self, x):
            return self.conv(tr_parallel(x, self.sf, self.db, self.dt))

    cpu = copy.deepcopy(model_fp).cpu().float().eval()
    qmods = dict(qmodel.named_modules())
    for name, m in list(cpu.named_modules()):
        if name in qmods and isinstance(qmods[name], tr_layer.TRConv2dLayer):
            parent = cpu
            keys = name.split(".")
            for k in keys[:-1]:
                parent = parent._modules[k]
            parent._modules[keys[-1]] = OracleTRConv(qmods[name])
    nthreads = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        x = util.SyntheticImageNet(nimg, nimg, seed=7).batch(0)[0]
        with torch.no_grad():
            cpu(x[:2])  # warm the allocator and the pool
            t0 = time.perf_counter()
            cpu(x)
            dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(nthreads)
        pool.shutdown()
    return {"value": nimg / dt, "unit": "images/s", "cores": threads, "kind": "port",
            "nproc": nproc, "cpu_model": cpu_model,
            "sample": "%d synthetic 3x224x224 images, ResNet-18 TQ forward: oracle TR "
                      "(oracle/tr_oracle.c) on every TR-layer activation split over %d threads + "
                      "torch-CPU fp32 conv (%d threads) on the fake-quantized tensors; weight TR "
                      "excluded (one-time conversion)" % (nimg, threads, threads),
            "tr_op": cpu_tr_op_baseline(oracle),
            "python_restatements": cpu_python_baselines(oracle)}


def cpu_python_baselines(oracle, nq=200000, nx=1 << 16):
    """BASELINE.md C1 and C2 on one core: the pure-Python restatements of bit_utils.hese
    (random q in [-511, 511], seed 0) and of the whole tr() (hese + the greedy group top-k,
    g=8, k=12, on relu(N(0,1)) fp32 at sf=0.05, db=9) -- oracle.hese_py / oracle.tr_py, the
    latter checked bit for bit against the C restatement on its sample here."""
    rng = np.random.default_rng(0)
    qs = rng.integers(-511, 512, nq).tolist()
    t0 = time.perf_counter()
    for q in qs:
        oracle.hese_py(q)
    t_hese = time.perf_counter() - t0
    x = np.maximum(rng.standard_normal(nx, dtype=np.float32), 0)
    t0 = time.perf_counter()
    y = oracle.tr_py(x, 0.05, DB, 8, 12)
    t_tr = time.perf_counter() - t0
    ok = bool(np.array_equal(y.view(np.int32),
                             oracle.tr(x.reshape(1, -1), 0.05, DB, 8, 12).reshape(-1).view(np.int32)))
    return {"c1_hese_values_per_s": nq / t_hese, "c2_tr_elements_per_s": nx / t_tr,
            "cores": 1, "kind": "port", "c2_matches_c_restatement": ok,
            "sample": "C1: %d random q in [-511, 511] (seed 0), oracle.hese_py; C2: %d relu(N(0,1)) "
                      "fp32, g=8 k=12 sf=0.05 db=%d, oracle.tr_py" % (nq, nx, DB),
            # C1 times the restatement; the reference's own encoder (bit_utils.hese,
            # bit_utils.py:10-44) cannot travel to the GPU box and is timed in the build
            # container on the same sample by tools/ref/time_ref_hese.py
            "c1_is": "restatement (oracle.hese_py), not the reference's bit_utils.hese",
            "c1_reference_encoder": "profiles/r06_ref_hese_cpu.txt"}


def cpu_tr_op_baseline(oracle, n=1 << 24):
    """SURVEY 8(d) CPU baseline (iii): the TR op alone (D1: relu(N(0,1)) activations,
    sf=0.05, db=9, dt=3, g=1) by the C oracle on 1 thread and on T host threads (chunks of the
    flat tensor; elements are independent at g=1 and ctypes releases the GIL), elements/s.
    T = OMP_NUM_THREADS (16 on the GPU box: its CPU share), else the visible core count.
    Beside it, the product's own host TR op (libtq_host.so, OpenMP, T threads)."""
    from concurrent.futures import ThreadPoolExecutor
    _, _, threads = host_info()
    x = np.maximum(np.random.default_rng(0).standard_normal(n, dtype=np.float32), 0)

    def run(chunk):
        return oracle.tr(chunk.reshape(1, -1, 1, 1), 0.05, DB, 1, DT)

    small = x[: n // 8]
    t0 = time.perf_counter()
    run(small)
    t1 = time.perf_counter() - t0
    chunks = np.array_split(x, threads * 4)
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(run, chunks[:threads]))  # warm the pool
        t0 = time.perf_counter()
        list(ex.map(run, chunks))
        tn = time.perf_counter() - t0
    host = None
    try:
        import tq_native
        xt = torch.from_numpy(x).view(1, -1, 1, 1)
        out = torch.empty_like(xt)
        nt = torch.get_num_threads()
        torch.set_num_threads(threads)
        try:
            tq_native.tr_into_host(xt, out, 0.05, DB, 1, DT)  # warm
            t0 = time.perf_counter()
            tq_native.tr_into_host(xt, out, 0.05, DB, 1, DT)
            host = n / (time.perf_counter() - t0)
        finally:
            torch.set_num_threads(nt)
    except Exception:  # noqa: BLE001 -- the host library is optional here
        host = None
    return {"elements_per_s_1thread": small.size / t1, "elements_per_s": n / tn,
            "threads": threads, "kind": "port",
            "sample": "%d relu(N(0,1)) fp32 elements, TR g=1 (sf=0.05, db=9, dt=3), "
                      "oracle/tr_oracle.c" % n,
            "product_host_tr_elements_per_s": host}


def d1_tr_op(dev, iters=20):
    """the TR op alone on the ResNet-18 layer-1 activation tensor,
    relu(N(0,1)) 256x64x56x56 fp32 (seed 0), sf=0.05, db=9, dt=3, g=1, viewed (1,-1,1,1) as
    tr_layer.py:96-99 calls it; 8 algorithmic bytes per element (fp32 read + write), HIP
    events on the launch stream, against the 8 TB/s HBM peak."""
    import tq_native
    torch.manual_seed(0)
    x = torch.relu(torch.randn(256, 64, 56, 56, device=dev)).view(1, -1, 1, 1)
    out = torch.empty_like(x)
    run = lambda: tq_native.tr_into(x, out, 0.05, DB, 1, DT)  # noqa: E731
    for _ in range(3):
        run()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(iters):
        run()
    b.record(s)
    torch.cuda.synchronize()
    t = a.elapsed_time(b) * 1e-3 / iters
    n = x.numel()
    gbs = 8 * n / t / 1e9
    return {"kernel": "tr_elem_kernel<float> (g=1: quantize + closed-form HESE + keep dt terms "
                      "+ rescale)", "elements": n, "us_per_launch": t * 1e6,
            "elements_per_s": n / t, "achieved_gbs": gbs, "peak_gbs": HBM_PEAK_GBS,
            "hbm_frac": gbs / HBM_PEAK_GBS, "bytes_per_element": 8, "launches": iters}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    what, val = launch_plan(args.gpus, os.environ)
    if what == "error":
        print("bench.py: " + val, file=sys.stderr)
        return 2
    if what == "spawn":
        return spawn_ranks(argv, val, args.dry_launch)
    world = val
    rank = int(os.environ.get("RANK", "0"))
    if args.dry_launch:
        print(json.dumps({"rank": rank, "world_size": world,
                          "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}))
        return 0
    os.environ["TQ_CONV_ENGINE"] = args.engine
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not check_world(world, local):
        return 2
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    torch.backends.cudnn.benchmark = True  # MIOpen picks its fastest stem-conv solver once
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    model_fp, qmodel, tmacs_per_img = build_model(dev, args.batch, rank)
    runner = qmodel if args.unfused else tq_fuse.FusedResNet(qmodel, stem=args.stem)

    # resident synthetic inputs (two batches, alternated) and labels
    data = util.SyntheticImageNet(2 * args.batch, args.batch, seed=rank, device=dev)
    batches = []
    for i in range(2):
        x, y = data.batch(i)
        batches.append((x.to(memory_format=torch.channels_last).contiguous(
            memory_format=torch.channels_last), y))
    counters = torch.zeros(2, dtype=torch.int64, device=dev)

    streams = None
    if args.streams > 1 and not args.unfused:
        streams = [torch.cuda.Stream(dev) for _ in range(args.streams)]

    def timed_steps(runner):
        """W untimed warmup steps, (optionally) one hipGraph per resident batch, then the K
        timed steps between barrier + synchronize: (seconds, launch mode, counters)."""
        def step(i):
            x, y = batches[i % 2]
            out = runner(x) if streams is None else runner.forward_streams(x, streams)
            counters[0] += (out.argmax(1) == y).sum()
            counters[1] += y.numel()

        for i in range(args.warmup):
            step(i)
        torch.cuda.synchronize()
        # --graph: one hipGraph per resident batch; the whole forward (stem conv, fused
        # term-pair convs, pooling, fc, counters) replays without per-kernel host launches.
        graphs, launch = None, "eager"
        if args.graph or args.launch == "graph":
            try:
                graphs = []
                for i in range(2):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        step(i)
                    graphs.append(g)
                launch = "hipGraph"
            except Exception as e:  # noqa: BLE001 -- reported in the JSON line
                graphs, launch = None, "eager (graph capture failed: %s)" % str(e)[:120]
                torch.cuda.synchronize()
        counters.zero_()

        def run(i):
            if graphs is not None:
                graphs[i % 2].replay()
            else:
                step(i)

        for i in range(2):  # graph upload / first replay outside the timed region
            run(i)
        counters.zero_()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for i in range(args.steps):
            run(i)
        if world > 1:
            dist.all_reduce(counters)  # the one collective: accuracy counters
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0, launch, [int(v) for v in counters.tolist()]

    with torch.no_grad():
        elapsed, launch, acc_counters = timed_steps(runner)

        # Kernel roofline pass: the same K steps again, eager, with HIP events around every
        # TQ kernel on its launch stream (events between kernels cost ~10 us of idle GPU
        # each, so they stay out of the timed region above).
        # The kernels are timed in isolation: one stream, full-batch launches (with chunk
        # streams two launches share the GPU, and a launch's duration no longer measures the
        # kernel -- the timed region's overlap is an executor-level gain, reported in value).
        timer = KernelTimer()
        tq_ops.set_kernel_hook(timer)
        pass_end = torch.cuda.Event(enable_timing=True)
        for i in range(args.steps):
            runner(batches[i % 2][0])
        pass_end.record(torch.cuda.current_stream())
        torch.cuda.synchronize()
        tq_ops.set_kernel_hook(None)
        # GPU time of that one-stream pass (its kernels plus the event gaps between them)
        roof_pass_s = timer.base.elapsed_time(pass_end) * 1e-3

        # the other stems: the same executor with the torch
        # fp32 stem conv (MIOpen, true fp32) + the BN/ReLU/max-pool/codes kernel, and with the
        # fused stem kernel with / without its exact fix-up, timed the same way, reported
        # beside the headline
        stem_legs = {}
        if world == 1 and not args.unfused and not args.no_stem_leg:
            for other in ("fp32", "exact", "fused"):
                if other == args.stem:
                    continue
                el2, launch2, _ = timed_steps(tq_fuse.FusedResNet(qmodel, stem=other))
                stem_legs["stem_" + other] = {
                    "stem": STEM_NAMES[other], "images_per_s": args.batch * args.steps / el2,
                    "ms_per_step": el2 / args.steps * 1e3, "launch": launch2,
                    "streams": args.streams}

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    images = args.batch * args.steps * world
    ips = images / elapsed
    kt = timer.summary()

    result = None
    if rank == 0:
        conv = kt["conv2d_termpair"]
        # the HBM-bound TR stage of the step: the fused stem tail (BN/ReLU/max-pool + the
        # first TR layer's activation TR) in the fused executor, act_encode otherwise
        enc_name = next(k for k in ("stem_conv_pool", "stem_pool_encode", "act_encode")
                        if k in kt)
        enc = kt[enc_name]
        # time per launch = the kernels' busy time / launches (the union of the launch
        # intervals: on the roofline pass's one stream it equals the summed durations,
        # avg_launch_us, which rocprofv3 --kernel-trace of a one-stream run reports)
        conv_t = conv["busy"] / conv["launches"]
        conv_work = conv["work"] / conv["launches"]
        enc_t = enc["busy"] / enc["launches"]
        enc_bytes = enc["work"] / enc["launches"]
        traffic = enc_traffic = None
        mfma = args.engine == "mfma"
        pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc_path):
            pmc = json.load(open(pmc_path))
            traffic = pmc.get("conv2d_tp_mfma_bytes_per_launch" if mfma else
                              "conv2d_tp_bytes_per_launch")
            enc_traffic = pmc.get(enc_name + "_bytes_per_launch")
        if mfma:
            roof = {
                "kernel": "conv2d_tp_mfma_kernel (term-pair conv, exact fp16 term sums, "
                          "v_mfma_f32_32x32x16_f16, int32 sums)",
                "bound": "mfma",
                "achieved": 2 * conv_work / conv_t / 1e12,
                "peak": MFMA_F16_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": 2 * conv_work / conv_t / 1e12 / MFMA_F16_PEAK_TFLOPS,
            }
        else:
            roof = {
                "kernel": "conv2d_tp_kernel (term-pair conv, int16 term sums, v_dot2c_i32_i16)",
                "bound": "valu",
                "achieved": conv_work / conv_t / 1e12,
                "peak": DOT2_PEAK / 1e12,
                "unit": "TMAC/s (int16 term-sum products)",
                "frac": conv_work / conv_t / DOT2_PEAK,
            }
        conv_bytes = conv["bytes"] / conv["launches"]
        roof.update({
            "traffic": traffic,
            "algorithmic_macs_per_launch": conv_work,
            # the tensors a conv launch reads/writes once (codes in, weight codes, fp32
            # residual / output, next layers' codes), beside the PMC-measured traffic
            "algorithmic_bytes_per_launch": conv_bytes,
            "achieved_gbs": conv_bytes / conv_t / 1e9,
            "avg_launch_us": conv["seconds"] / conv["launches"] * 1e6,
            "busy_us_per_launch": conv_t * 1e6,
            "launches": conv["launches"],
            # like for like: the convs' busy time over the GPU time of the same one-stream
            # roofline pass (both include the ~10 us event gaps' absence / presence alike)
            "share_of_roofline_pass": conv["busy"] / roof_pass_s,
            "roofline_pass_ms_per_step": roof_pass_s / args.steps * 1e3,
            # the north star's HBM roofline of the whole path: 15,026,432
            # algorithmic bytes per image (fp32 TR-layer inputs + outputs + weights/256) at
            # the measured images/s against the 8 TB/s HBM peak
            # per-launch roofline: each launch's bound is the larger of its MFMA time
            # (2 * MACs / fp16 peak) and its HBM time (algorithmic bytes / 8 TB/s); the
            # sum of those floors over the convs' summed launch durations (layer-1/2 convs
            # and every fp32-residual conv2 sit on the HBM side of the ridge)
            "per_launch_bound_frac": (sum(max(2 * w / (MFMA_F16_PEAK_TFLOPS * 1e12),
                                               nb / (HBM_PEAK_GBS * 1e9))
                                           for w, nb in conv["per_launch"]) / conv["seconds"]
                                      if mfma else None),
            "per_launch_hbm_bound_launches": (sum(
                1 for w, nb in conv["per_launch"]
                if nb / (HBM_PEAK_GBS * 1e9) > 2 * w / (MFMA_F16_PEAK_TFLOPS * 1e12))
                if mfma else None),
            "hbm_bytes_per_image": HBM_BYTES_PER_IMAGE,
            "hbm_frac": HBM_BYTES_PER_IMAGE * ips / (HBM_PEAK_GBS * 1e9),
        })
        if enc_name == "stem_conv_pool":
            # the fused stem: near-fp32 conv on split-fp16 MFMAs + BN/ReLU/pool + codes;
            # algorithmic work = the reference's fp32 conv MACs, priced against the fp32
            # peak (the arithmetic the reference runs, 157.3 TFLOP/s MFMA/VALU)
            n_img = args.batch  # images per launch (the roofline pass is one stream)
            stem_bytes = n_img * (3 * 224 * 224 * 4 + 64 * 56 * 56 * (4 + 2))
            roof_tr = {
                "kernel": "stem_conv_pool_kernel (ResNet stem conv 7x7/2 in near-fp32 arithmetic "
                          "on split-fp16 v_mfma_f32_16x16x32_f16 + BN/ReLU/max-pool + first "
                          "activation TR -> fp16 codes)" + (
                              " + stem_fixup_kernel (exact fp64 recompute of the listed "
                              "near-midpoint outputs; time included)"
                              if args.stem == "exact" else ""),
                "bound": "mfma",
                # what the matrix cores execute: 3 fp16 split products per fp32 MAC, against
                # the dense fp16 MFMA peak
                "achieved": 3 * 2 * enc_bytes / enc_t / 1e12,
                "peak": MFMA_F16_PEAK_TFLOPS,
                "unit": "TFLOP/s (fp16 MFMA, 3 split products per fp32 MAC)",
                "frac": 3 * 2 * enc_bytes / enc_t / 1e12 / MFMA_F16_PEAK_TFLOPS,
                "hbm_gbs": stem_bytes / enc_t / 1e9,
                # secondary: the reference's fp32 conv MACs priced against the fp32 peak
                "fp32_equiv_tflops": 2 * enc_bytes / enc_t / 1e12,
                "fp32_equiv_frac": 2 * enc_bytes / enc_t / 1e12 / FP32_PEAK_TFLOPS,
                "traffic": enc_traffic,
                "algorithmic_macs_per_launch": enc_bytes,
                "avg_launch_us": enc["seconds"] / enc["launches"] * 1e6,
                "busy_us_per_launch": enc_t * 1e6,
                "launches": enc["launches"],
            }
        else:
            roof_tr = {
                "kernel": ("bn_relu_maxpool_encode_kernel (stem BN/ReLU/max-pool + activation "
                           "TR -> 16-bit codes)" if enc_name == "stem_pool_encode" else
                           "act_encode_kernel (TR of activations -> 16-bit codes)"),
                "bound": "hbm",
                "achieved": enc_bytes / enc_t / 1e9,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": enc_bytes / enc_t / 1e9 / HBM_PEAK_GBS,
                "traffic": enc_traffic,
                "algorithmic_bytes_per_launch": enc_bytes,
                "avg_launch_us": enc_t * 1e6,
                "launches": enc["launches"],
            }
        result = {
            "metric": METRIC,
            "value": ips,
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            # exact integer term-pair sums: codes are integers held in fp16 (MFMA engine) or
            # int16 (VALU engine), products exact in fp32, sums flushed to int32
            "dtype": "int (exact, fp16-coded)" if mfma else "int (exact, int16-coded)",
            "data": "synthetic",
            "config": {"workload": "resnet18-tq-g8-k12 (wb=db=9, dt=3), synthetic N(0,1) "
                                   "3x224x224, random-init weights",
                       "per_gpu_batch": args.batch, "global_batch": args.batch * world,
                       "parallelism": "dp%d (batch-sharded, no data-path collective)" % world,
                       "engine": args.engine,
                       "executor": "module path" if args.unfused else
                                   "fused (BN/ReLU/residual/next-layer TR in the conv "
                                   "epilogue)",
                       "launch": launch, "streams": args.streams,
                       # the stem conv (not a TR layer; fp32 torch in the reference) runs in
                       # the fused stem kernel as a split-fp16 conv with the exact fix-up
                       # (default: correctly rounded codes), without it (--stem fused), or
                       # (--stem fp32) as torch's fp32 conv
                       "stem": STEM_NAMES[args.stem if enc_name == "stem_conv_pool" else "fp32"]},
            "term_pair_macs_per_image": tmacs_per_img,
            "term_pair_macs_per_s": tmacs_per_img * ips,
            "roofline": roof,
            "roofline_tr": roof_tr,
            "accuracy_counters": acc_counters,
        }
        result.update(stem_legs)
        if world == 1 and not args.no_d1:
            result["d1_tr_op"] = d1_tr_op(dev)
        if world == 1 and not args.no_d4:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import bench_d4
            result["d4"] = bench_d4.d4_summary(dev)
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(model_fp, qmodel, args.cpu_sample)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if result is not None:
        print(json.dumps(result))
    return 0


if __name__ == "__main__":
    sys.exit(main())
