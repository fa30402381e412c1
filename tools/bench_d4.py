"""the other configs of BASELINE.json on one MI355X, one JSON line each.

    python tools/bench_d4.py [--steps 10]

* LSTM-650 Wikitext-2 TQ (g=8, k=12, wb=db=dt=8), eval batch 10, bptt 35: random-init
  RNNModel and uniform random token ids (the WikiText-2 train split that defines the
  vocabulary is not available offline; the vocabulary size 33,278 is kept).  tokens/s of the
  TQ forward (TR'd LSTM weights + quantized inputs/hidden state at chunk boundaries, the
  reference's TRLSTMLayer semantics) and term-pair MACs/s with the decoder count of
  profile_model (as published).
* MobileNet-V2 / EfficientNet-b0 TQ (depthwise layers at wb=16, g=1, k=16 as
  cnn_models.static_conv_layer_settings sets them; other layers g=8, k=12, wb=db=9, dt=3),
  synthetic N(0,1) 256x3x224x224, random-init weights: images/s of the converted module path
  (term-pair and depthwise term-pair kernels, torch BN/activations), and for MobileNet-V2
  also of the fused executor (tq_fuse.FusedMobileNetV2: BN / ReLU6 / residual / next-layer
  TR in the kernels' epilogues).
Timing: W untimed warmup steps, then K steps between synchronize calls."""
import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))

import cnn_models  # noqa: E402
import evaluate_lstm  # noqa: E402
import profile_model  # noqa: E402
import tq_fuse  # noqa: E402
import tq_ops  # noqa: E402
import tr_layer  # noqa: E402
from lstm_models import model as model_mod  # noqa: E402

sys.path.insert(0, ROOT)
from bench import HBM_PEAK_GBS, MFMA_F16_PEAK_TFLOPS, KernelTimer  # noqa: E402

# MI355X_MICROARCH.md: a 38 MB table read from the Infinity Cache at 8.6 TB/s chip-wide
# ("Indexed rows: gather into LDS"); a dependent kernel boundary on one stream 1.45 us between
# trivial kernels ("boundary" row, eager = hipGraph)
MALL_GATHER_GBS = 8600.0
KERNEL_BOUNDARY_US = 1.45

FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: fp32 vector = fp32 matrix peak


def kernel_breakdown(fn, steps, total_s):
    """A second pass of `steps` steps with HIP events around every TQ kernel (tq_ops hook, as
    bench.py): per kernel family launches, average duration, share of the step and its
    roofline -- term-pair MFMA convs against the dense fp16 MFMA peak (2 FLOP per term-sum
    product), the HBM-bound kernels (activation encode, depthwise) against 8 TB/s with
    their algorithmic bytes."""
    timer = KernelTimer()
    tq_ops.set_kernel_hook(timer)
    try:
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
    finally:
        tq_ops.set_kernel_hook(None)
    out = {}
    for name, k in timer.summary().items():
        e = {"launches_per_step": k["launches"] // steps,
             "avg_launch_us": k["seconds"] / k["launches"] * 1e6,
             "share_of_step": k["seconds"] / steps / total_s}
        if name == "conv2d_termpair":
            tf = 2 * k["work"] / k["seconds"] / 1e12
            e.update({"bound": "mfma", "achieved_tflops": tf, "peak_tflops": MFMA_F16_PEAK_TFLOPS,
                      "frac": tf / MFMA_F16_PEAK_TFLOPS})
            if k["bytes"]:  # fused convs state their algorithmic bytes: the HBM side too
                gbs = k["bytes"] / k["seconds"] / 1e9
                e.update({"achieved_gbs": gbs, "peak_gbs": HBM_PEAK_GBS,
                          "hbm_frac": gbs / HBM_PEAK_GBS})
        elif name in ("act_encode", "act_encode_act"):
            gbs = k["work"] / k["seconds"] / 1e9
            e.update({"bound": "hbm", "achieved_gbs": gbs, "peak_gbs": HBM_PEAK_GBS,
                      "frac": gbs / HBM_PEAK_GBS})
        else:  # depthwise / wide term-pair kernels: work = term-sum products
            e.update({"term_sum_macs_per_s": k["work"] / k["seconds"]})
            if k["bytes"]:  # depthwise: HBM-bound (codes in, fp32 out, once each)
                gbs = k["bytes"] / k["seconds"] / 1e9
                e.update({"bound": "hbm", "achieved_gbs": gbs, "peak_gbs": HBM_PEAK_GBS,
                          "frac": gbs / HBM_PEAK_GBS})
        out[name] = e
    return out


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def timed_median(fn, steps, warmup, reps=3):
    """Median over `reps` back-to-back timed loops of `steps` steps (one host hiccup in an
    eager launch loop of ~100 launches per step otherwise moves a short loop's mean)."""
    ts = [timed(fn, steps, warmup if i == 0 else 0) for i in range(reps)]
    return sorted(ts)[len(ts) // 2]


def timed_graph(fn, steps, warmup):
    """fn captured once as a hipGraph and replayed (no per-kernel host launches); None when
    the capture fails."""
    try:
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        g.replay()
        torch.cuda.synchronize()
    except Exception:  # noqa: BLE001 -- reported as None
        torch.cuda.synchronize()
        return None
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


class _Segments(object):
    """HIP events around named segments of a forward on the current stream (a second,
    instrumented pass: the events between kernels add a little idle time, so the shares are
    of the instrumented step)."""

    def __init__(self):
        self.ev = []

    def wrap(self, name, fn):
        def run(*a, **k):
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            r = fn(*a, **k)
            e1.record(s)
            self.ev.append((name, e0, e1))
            return r
        return run

    def totals(self):
        out = {}
        for name, e0, e1 in self.ev:
            out[name] = out.get(name, 0.0) + e0.elapsed_time(e1) * 1e-3
        return out


def lstm_breakdown(qt, model, x, hidden, steps):
    """Where the term-pair LSTM-650 chunk's time goes (BASELINE configs[2]): the instrumented
    forward's kernel families -- the layer-0 input projection (TR(emb) encode + the term-pair
    GEMM, tq_ops.tr_linear), the two recurrences in wavefront order (tq_lstm_seq2_f32: T + 1
    launches of lstm_step2_kernel), the fp32 decoder (torch Linear, the reference's
    TRLinearLayer semantics: the unquantized input) and log_softmax -- each with its share of
    the instrumented step and its roofline."""
    import tq_native
    seg = _Segments()
    saved = (tq_native.lstm_seq2, tq_ops.tr_linear, qt.decoder.forward)
    tq_native.lstm_seq2 = seg.wrap("recurrence", saved[0])
    tq_ops.tr_linear = seg.wrap("input_projection", saved[1])
    qt.decoder.forward = seg.wrap("decoder", saved[2])
    import torch.nn.functional as F
    lsm = F.log_softmax
    F.log_softmax = seg.wrap("log_softmax", lsm)
    try:
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(steps):
            qt(x, hidden)
        e1.record(s)
        torch.cuda.synchronize()
    finally:
        tq_native.lstm_seq2, tq_ops.tr_linear = saved[0], saved[1]
        qt.decoder.forward = saved[2]
        F.log_softmax = lsm
    step = e0.elapsed_time(e1) * 1e-3 / steps
    tot = {k: v / steps for k, v in seg.totals().items()}
    T, B = x.shape
    H, V = model.nhid, model.ntoken
    D = model.encoder.embedding_dim
    fam = {}
    if "recurrence" in tot:
        launches = T + 1
        # bytes a launch must read: W_hh0, W_ih1, W_hh1 (fp32 [4H][H] each; launch s runs layer
        # 0's step s and layer 1's step s - 1), 20.3 MB -- resident in the 256 MB Infinity
        # Cache (MALL) after the first step, so the floor of a launch is those bytes at the
        # resident-table read rate plus one dependent kernel boundary (the launches form a
        # chain: each step needs the previous one's h, c); the HBM figure is kept beside it
        wbytes = 3 * 4 * H * H * 4
        per = tot["recurrence"] / launches
        floor = wbytes / (MALL_GATHER_GBS * 1e9) + KERNEL_BOUNDARY_US * 1e-6
        fam["lstm_step2_kernel"] = {
            "launches_per_step": launches, "avg_launch_us": per * 1e6,
            "share_of_step": tot["recurrence"] / step, "bound": "mall+latency",
            "bytes_per_launch": wbytes, "achieved_gbs": wbytes / per / 1e9,
            "peak_gbs": MALL_GATHER_GBS, "floor_us_per_launch": floor * 1e6,
            "frac": floor / per,
            "hbm_frac": wbytes / per / 1e9 / HBM_PEAK_GBS}
    if "input_projection" in tot:
        prods = T * B * D * 4 * H
        tf = 2 * prods / tot["input_projection"] / 1e12
        fam["input_projection"] = {
            "what": "TR(emb) codes + term-pair GEMM %dx%d -> %d (MFMA engine)" % (
                T * B, D, 4 * H),
            "avg_us": tot["input_projection"] * 1e6,
            "share_of_step": tot["input_projection"] / step, "bound": "mfma",
            "achieved_tflops": tf, "peak_tflops": MFMA_F16_PEAK_TFLOPS,
            "frac": tf / MFMA_F16_PEAK_TFLOPS}
    if "decoder" in tot:
        tf = 2 * T * B * H * V / tot["decoder"] / 1e12
        fam["decoder_fp32"] = {
            "what": "torch fp32 Linear %d -> %d on %d rows (reference semantics)" % (H, V, T * B),
            "avg_us": tot["decoder"] * 1e6, "share_of_step": tot["decoder"] / step,
            "bound": "fp32", "achieved_tflops": tf, "peak_tflops": FP32_PEAK_TFLOPS,
            "frac": tf / FP32_PEAK_TFLOPS}
    if "log_softmax" in tot:
        nb = 2 * T * B * V * 4
        fam["log_softmax"] = {
            "avg_us": tot["log_softmax"] * 1e6, "share_of_step": tot["log_softmax"] / step,
            "bound": "hbm", "bytes": nb, "achieved_gbs": nb / tot["log_softmax"] / 1e9,
            "peak_gbs": HBM_PEAK_GBS, "frac": nb / tot["log_softmax"] / 1e9 / HBM_PEAK_GBS}
    rest = step - sum(tot.values())
    fam["other"] = {"what": "embedding, h0/c0 TR, copies, launch gaps", "avg_us": rest * 1e6,
                    "share_of_step": rest / step}
    return {"instrumented_step_ms": step * 1e3, "families": fam}


def lstm(args, dev):
    torch.manual_seed(1111)
    ntokens, bsz, bptt = evaluate_lstm.WT2_VOCAB, 10, 35
    model = model_mod.RNNModel("LSTM", ntokens, 650, 650, 2, 0.5, True).to(dev).eval()
    tr_params = evaluate_lstm.static_lstm_layer_settings(model, 8, 8, 12)
    q = evaluate_lstm.convert_model(model, tr_params, 8, 8, termpair=False)
    tokens = torch.randint(0, ntokens, (bptt * bsz * 4 + bsz,))
    data = evaluate_lstm.batchify(tokens, bsz, dev)
    x = evaluate_lstm.get_batch(data, 0, bptt)[0]
    with torch.no_grad():
        q(x, model.init_hidden(bsz))  # calibration pass
        tr_layer.set_tr_tracking(q, False)
        tmacs, _ = profile_model.get_model_ops(q, inputs=(x, model.init_hidden(bsz)))
        hidden = model.init_hidden(bsz)
        t = timed(lambda: q(x, hidden), args.steps, args.warmup)
        # the same model with TRLSTMLayer(termpair=True) (the default): layer 0 on the
        # term-pair kernels; `value` stays the MIOpen composition for comparability
        qt = evaluate_lstm.convert_model(model, tr_params, 8, 8, termpair=True)
        qt(x, model.init_hidden(bsz))
        tr_layer.set_tr_tracking(qt, False)
        t_tp = timed(lambda: qt(x, hidden), args.steps, args.warmup)
        breakdown = lstm_breakdown(qt, model, x, hidden, args.steps)
        # the decoder as a term-pair GEMM (TRLinearLayer(quantize_input=True): linear(TR(h),
        # TR(W)) on the MFMA engine), timed alone on the 350 x 650 LSTM output -- not on the
        # timed path (the reference's TRLinearLayer runs the dense layer on the unquantized
        # input), reported as the secondary term-pair line
        dec = torch.nn.Linear(650, ntokens).to(dev)
        dec.weight.data.copy_(model.decoder.weight.data)
        dec.bias.data.copy_(model.decoder.bias.data)
        tpl = tr_layer.TRLinearLayer(dec, 8, 8, 8, 8, 12, quantize_input=True)
        h = torch.randn(bptt * bsz, 650, device=dev).tanh()
        tpl(h)
        tpl.tracking(False)
        td = timed(lambda: tpl(h), args.steps, args.warmup)
    toks = bptt * bsz
    dec_macs = toks * 650 * ntokens
    return {"metric": "LSTM-650 TQ tokens/s", "value": toks / t, "unit": "tokens/s",
            "ms_per_step": t * 1e3,
            # profile_model's count (the published metric) is analytic: this forward keeps the
            # reference's semantics (TRLSTMLayer: fp32 MIOpen LSTM on TR'd weights / quantized
            # inputs; TRLinearLayer: dense decoder on the unquantized input), no term-pair kernel
            "analytic_term_pair_macs_per_step": tmacs,
            "analytic_term_pair_macs_per_s": tmacs / t,
            "termpair_lstm_tokens_per_s": toks / t_tp,
            "termpair_breakdown": breakdown,
            "term_pair_decoder": {
                "what": "TRLinearLayer(quantize_input=True) 650 -> %d on %d rows, term-pair "
                        "GEMM on the MFMA engine, timed alone" % (ntokens, toks),
                "ms": td * 1e3, "term_sum_products": dec_macs,
                "achieved_tflops": 2 * dec_macs / td / 1e12,
                "frac_of_fp16_mfma_peak": 2 * dec_macs / td / 1e12 / MFMA_F16_PEAK_TFLOPS},
            "config": {"workload": "lstm-650 wikitext-2 vocab, g=8 k=12 wb=db=dt=8",
                       "batch": bsz, "bptt": bptt, "data": "synthetic token ids"}}


def lstm_trace(chunks, dev):
    """Profiling mode (tools/gpu_lstm_trace.sh): the term-pair LSTM-650 model of lstm() alone,
    calibrated and warmed, then `chunks` 350-token forwards between synchronize calls; prints
    the host clocks around them so tools/trace_window.py can cut exactly those chunks out of a
    rocprofv3 kernel trace."""
    torch.manual_seed(1111)
    ntokens, bsz, bptt = evaluate_lstm.WT2_VOCAB, 10, 35
    model = model_mod.RNNModel("LSTM", ntokens, 650, 650, 2, 0.5, True).to(dev).eval()
    tr_params = evaluate_lstm.static_lstm_layer_settings(model, 8, 8, 12)
    tokens = torch.randint(0, ntokens, (bptt * bsz * 4 + bsz,))
    x = evaluate_lstm.get_batch(evaluate_lstm.batchify(tokens, bsz, dev), 0, bptt)[0]
    with torch.no_grad():
        qt = evaluate_lstm.convert_model(model, tr_params, 8, 8, termpair=True)
        hidden = model.init_hidden(bsz)
        qt(x, hidden)  # calibration pass
        tr_layer.set_tr_tracking(qt, False)
        for _ in range(3):
            qt(x, hidden)
        torch.cuda.synchronize()
        clocks = {"monotonic": time.CLOCK_MONOTONIC, "boottime": time.CLOCK_BOOTTIME}
        w0 = {k: time.clock_gettime_ns(c) for k, c in clocks.items()}
        t0 = time.perf_counter()
        for _ in range(chunks):
            qt(x, hidden)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / chunks
        w1 = {k: time.clock_gettime_ns(c) for k, c in clocks.items()}
    return {"chunks": chunks, "tokens_per_chunk": bptt * bsz, "ms_per_chunk": t * 1e3,
            "tokens_per_s": bptt * bsz / t, "window_ns": {k: [w0[k], w1[k]] for k in w0}}


def cnn(arch, args, dev):
    torch.manual_seed(0)
    model = getattr(cnn_models, arch)(pretrained=False).to(dev).eval()
    settings = cnn_models.static_conv_layer_settings(model, 9, 8, 12)
    q = cnn_models.convert_model(model, settings, 9, 3).to(memory_format=torch.channels_last)
    x = torch.randn(args.batch, 3, 224, 224, device=dev).contiguous(
        memory_format=torch.channels_last)
    with torch.no_grad():
        tmacs, _ = profile_model.get_model_ops(q, (torch.randn(1, 3, 224, 224, device=dev),))
        q(x)
        tr_layer.set_tr_tracking(q, False)
        t = timed(lambda: q(x), args.steps, args.warmup)
        kernels = kernel_breakdown(lambda: q(x), args.steps, t)
        fused = None
        if arch in ("mobilenet_v2", "efficientnet_b0"):  # fused executors (tq_fuse.py)
            ex = (tq_fuse.FusedMobileNetV2 if arch == "mobilenet_v2" else
                  tq_fuse.FusedEfficientNet)(q)
            tf1 = timed(lambda: ex(x), args.steps, args.warmup)
            streams = [torch.cuda.Stream() for _ in range(2)]
            tf = timed(lambda: ex.forward_streams(x, streams), args.steps, args.warmup)
            tg = timed_graph(lambda: ex(x), args.steps, args.warmup)
            fused = {"images_per_s": args.batch / tf, "ms_per_step": tf * 1e3,
                     "streams": 2, "images_per_s_one_stream": args.batch / tf1,
                     "term_pair_macs_per_s": tmacs * args.batch / tf,
                     # the same forward replayed as one hipGraph: with ~50 launches of
                     # ~100 us the eager loop is partly host-bound
                     "images_per_s_graph": args.batch / tg if tg else None,
                     "kernels": kernel_breakdown(lambda: ex(x), args.steps, tf)}
    modes = sorted({m.mode for m in q.modules() if isinstance(m, tr_layer.TRConv2dLayer)})
    return {"metric": "%s TQ images/s" % arch, "value": args.batch / t, "unit": "images/s",
            "ms_per_step": t * 1e3, "term_pair_macs_per_image": tmacs,
            "term_pair_macs_per_s": tmacs * args.batch / t,
            "config": {"workload": "%s-tq (dw wb=16 g=1 k=16; others g=8 k=12 wb=db=9 dt=3)"
                                   % arch, "batch": args.batch, "layer_modes": modes,
                       "data": "synthetic N(0,1), random-init weights"},
            "kernels": kernels, "fused_executor": fused}


def cnn_fused(arch, steps, warmup, batch, dev, nstreams=2):
    """The fused executor of a depthwise config alone (bench.py's d4 key): images/s and the
    per-kernel rooflines.  Every term-pair conv of these executors is a 1x1 conv with
    Cin <= 960 whose bytes outweigh its products (codes in, fp32/codes out), so it is priced
    against HBM, as the depthwise and encode kernels are."""
    torch.manual_seed(0)
    model = getattr(cnn_models, arch)(pretrained=False).to(dev).eval()
    settings = cnn_models.static_conv_layer_settings(model, 9, 8, 12)
    q = cnn_models.convert_model(model, settings, 9, 3).to(memory_format=torch.channels_last)
    x = torch.randn(batch, 3, 224, 224, device=dev).contiguous(
        memory_format=torch.channels_last)
    with torch.no_grad():
        q(x)
        tr_layer.set_tr_tracking(q, False)
        ex = (tq_fuse.FusedMobileNetV2 if arch == "mobilenet_v2" else
              tq_fuse.FusedEfficientNet)(q)
        tf1 = timed_median(lambda: ex(x), steps, warmup)
        streams = [torch.cuda.Stream() for _ in range(nstreams)]
        # image chunks on their own streams (tq_fuse forward_streams): the measured rate
        tf = timed_median(lambda: ex.forward_streams(x, streams), steps, warmup)
        # per-kernel rooflines from one-stream launches (concurrent launches share the GPU)
        kern = kernel_breakdown(lambda: ex(x), steps, tf1)
    tp = kern.get("conv2d_termpair")
    if tp is not None:  # 1x1 convs: HBM-bound (algorithmic bytes per launch, fused _Conv)
        tp.update({"bound": "hbm", "mfma_frac": tp.pop("frac"), "frac": tp.pop("hbm_frac", None)})
    dom = max(kern, key=lambda k: kern[k]["share_of_step"])
    # the executor's faster launch mode on this box (both are the same kernels and logits:
    # test_fused_*_stream_split_bit_identical); both rates are reported
    best, streams_used = (tf, nstreams) if tf <= tf1 else (tf1, 1)
    return {"images_per_s": batch / best, "ms_per_step": best * 1e3, "batch": batch,
            "streams": streams_used, "images_per_s_streams": batch / tf,
            "images_per_s_one_stream": batch / tf1,
            "timing": "median of 3 loops of %d eager steps each" % steps,
            "dominant_kernel": dom, "kernels": kern}


def d4_summary(dev, steps=10, warmup=3, batch=256):
    """BASELINE configs[2] and [3] on one GPU, compactly (bench.py's "d4" key): LSTM-650
    tokens/s (term-pair layer-0 path and the MIOpen composition) with the term-pair decoder
    GEMM's roofline; fused MobileNet-V2 / EfficientNet-b0 images/s with per-kernel rooflines."""
    a = argparse.Namespace(steps=steps, warmup=warmup, batch=batch)
    out = {}
    r = lstm(a, dev)
    fams = r["termpair_breakdown"]["families"]
    dom = max((k for k in fams if k != "other"), key=lambda k: fams[k]["share_of_step"])
    out["lstm650"] = {"tokens_per_s": r["termpair_lstm_tokens_per_s"],
                      "tokens_per_s_miopen_composition": r["value"],
                      # the timed path's kernel families; roofline = the dominant one's
                      "dominant_kernel": dom,
                      "roofline": dict(fams[dom], kernel=dom),
                      "families": fams,
                      "term_pair_decoder_alone": dict(
                          r["term_pair_decoder"], bound="mfma", peak_tflops=MFMA_F16_PEAK_TFLOPS,
                          frac=r["term_pair_decoder"]["frac_of_fp16_mfma_peak"],
                          on_timed_path=False),
                      "config": r["config"]}
    for arch in ("mobilenet_v2", "efficientnet_b0"):
        out[arch] = cnn_fused(arch, steps, warmup, batch, dev)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--only", choices=("lstm", "mobilenet_v2", "efficientnet_b0"),
                    help="run one config")
    ap.add_argument("--fused-only", choices=("mobilenet_v2", "efficientnet_b0"),
                    help="the fused executor of one config alone (profiling runs)")
    ap.add_argument("--streams", type=int, default=2, help="image chunks / streams (fused-only)")
    ap.add_argument("--lstm-trace", type=int, default=0, metavar="CHUNKS",
                    help="profiling mode: CHUNKS term-pair LSTM-650 chunks and their clocks")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = True
    if args.lstm_trace:
        print(json.dumps(lstm_trace(args.lstm_trace, dev)), flush=True)
        return
    if args.fused_only:
        print(json.dumps(cnn_fused(args.fused_only, args.steps, args.warmup, args.batch, dev,
                                   args.streams)), flush=True)
        return
    runs = [("lstm", lambda: lstm(args, dev)),
            ("mobilenet_v2", lambda: cnn("mobilenet_v2", args, dev)),
            ("efficientnet_b0", lambda: cnn("efficientnet_b0", args, dev))]
    for name, fn in runs:
        if args.only and name != args.only:
            continue
        r = fn()
        if not math.isfinite(r["value"]):
            raise RuntimeError("non-finite result")
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
