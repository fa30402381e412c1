"""Per-workgroup phase timing of one term-pair conv launch (direct engine), from the timing-only
build `bash tools/ab/variant.sh trace -DTQ_PHASE_TRACE=1` (s_memrealtime stamps at workgroup start,
main-loop end and epilogue end; select the build with TQ_LIB_PATH).

    TQ_LIB_PATH=$PWD/term-quantization_amd/lib/libtq_hip_trace.so \\
        python tools/phase_probe.py --layer 2 --codes 1 --residual
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import tq_native  # noqa: E402
import tq_ops  # noqa: E402
from microbench import RESNET18_TR, make_layer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", type=int, default=2)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--codes", type=int, default=1)
    ap.add_argument("--residual", action="store_true")
    ap.add_argument("--no-out", action="store_true")
    ap.add_argument("--shape", default=None, help="cin,cout,k,stride,hin instead of --layer")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cin, cout, k, s, hin = (RESNET18_TR[args.layer - 1] if args.shape is None else
                            tuple(int(v) for v in args.shape.split(",")))
    args.kc = None
    layer = make_layer(cin, cout, k, s, dev, args)
    cp = tq_ops.act_channels(cin)
    xi = torch.relu(torch.randn(args.batch, cin, hin, hin, device=dev)).to(
        memory_format=torch.channels_last)
    codes = torch.empty((args.batch, hin, hin, cp), dtype=layer.w_codes.dtype, device=dev)
    tq_native.act_encode(xi, True, 0.02, 9, 3, codes)
    ho = (hin + 2 * (k // 2) - k) // s + 1
    o = torch.empty((args.batch, cout, ho, ho), device=dev, memory_format=torch.channels_last)
    sc = torch.full((cout,), 1e-4, dtype=torch.float64, device=dev)
    sh = torch.zeros(cout, dtype=torch.float64, device=dev)
    res = torch.randn_like(o) if args.residual else None
    cpo = tq_ops.act_channels(cout)
    ca = torch.empty((args.batch, ho, ho, cpo), dtype=codes.dtype, device=dev) \
        if args.codes >= 1 else None
    q = (0.05, 9, 3)
    fn = lambda: tq_native.conv2d_termpair_fused(  # noqa: E731
        codes, layer.w_codes, cout, k, k, (s, s), (k // 2, k // 2), (1, 1), ho, ho,
        out=None if args.no_out else o, ch_scale=sc, ch_shift=sh, residual=res, relu=True,
        codes_a=ca, quant_a=q if ca is not None else None, config=10,
        kc_steps=layer.kc_steps, kc_chunk=getattr(layer, "kc_chunk", -1))
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    fn()
    torch.cuda.synchronize()
    nwg = (args.batch * ho * ho + 127) // 128 * ((cout + 63) // 64)  # config 10: 64 x 128 tiles
    nwg = min(nwg, 1 << 16)
    buf = np.zeros((nwg, 4), dtype=np.uint64)
    lib = tq_native.lib()
    lib.tq_phase_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert lib.tq_phase_trace_read(buf.ctypes.data, nwg) == 0
    t0, t1, t2 = (buf[:, i].astype(np.int64) for i in range(3))
    base = t0.min()
    t0, t1, t2 = (t0 - base) / 100.0, (t1 - base) / 100.0, (t2 - base) / 100.0  # us
    hw = buf[:, 3] & 0xffffffff
    xcc = buf[:, 3] >> np.uint64(32)
    cu = ((hw >> np.uint64(8)) & np.uint64(15)) | (((hw >> np.uint64(13)) & np.uint64(3)) << np.uint64(4))
    span = t2.max()
    life = t2 - t0
    loop = t1 - t0
    epi = t2 - t1
    print("layer %d: %d workgroups, span %.1f us" % (args.layer, nwg, span))
    for name, v in (("lifetime", life), ("setup+main loop", loop), ("epilogue", epi)):
        print("  %-16s mean %7.2f  p10 %7.2f  p50 %7.2f  p90 %7.2f us" % (
            name, v.mean(), *np.percentile(v, [10, 50, 90])))
    print("  avg workgroups alive %.0f (%.2f per CU); xcc ids %s; cu-ids seen %d" % (
        life.sum() / span, life.sum() / span / 256, sorted(set(xcc.tolist()))[:8],
        len(set(zip(xcc.tolist(), cu.tolist())))))
    # start-time histogram: how quickly the grid drains
    h, e = np.histogram(t0, bins=10, range=(0, span))
    print("  starts per decile of the span:", h.tolist())
    order = np.argsort(t0)
    print("  first 5 starts (us):", np.round(t0[order[:5]], 2).tolist(),
          " last start %.1f, last end %.1f" % (t0.max(), span))


if __name__ == "__main__":
    main()
