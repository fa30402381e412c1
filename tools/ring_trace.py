"""Per-tile phase timing of one tap-ring conv launch, from the timing-only build
`bash tools/ab/variant1.sh rtrace tr_conv_ring "-DRING_TRACE=1"` (wave 0's s_memrealtime stamps per
tile: start, first barrier passed, K loop done, epilogue issued; select it with TQ_LIB_PATH).

    TQ_LIB_PATH=$PWD/term-quantization_amd/lib/libtq_hip_rtrace.so \\
        python tools/ring_trace.py --layer 6 --residual
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
    ap.add_argument("--layer", type=int, default=6)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--residual", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cin, cout, k, s, hin = RESNET18_TR[args.layer - 1]
    args.kc = None
    args.nonneg = True
    layer = make_layer(cin, cout, k, s, dev, args)
    cp = tq_ops.act_channels(cin)
    xi = torch.relu(torch.randn(args.batch, cin, hin, hin, device=dev)).to(
        memory_format=torch.channels_last)
    codes = torch.empty((args.batch, hin, hin, cp), dtype=layer.w_codes.dtype, device=dev)
    tq_native.act_encode(xi, True, 0.02, 9, 3, codes)
    ho = hin
    o = torch.empty((args.batch, cout, ho, ho), device=dev, memory_format=torch.channels_last)
    sc = torch.full((cout,), 1e-4, dtype=torch.float64, device=dev)
    sh = torch.zeros(cout, dtype=torch.float64, device=dev)
    res = torch.randn_like(o) if args.residual else None
    ca = torch.empty((args.batch, ho, ho, tq_ops.act_channels(cout)), dtype=codes.dtype,
                     device=dev)
    fn = lambda: tq_native.conv2d_termpair_fused(  # noqa: E731
        codes, layer.w_codes, cout, k, k, (s, s), (k // 2, k // 2), (1, 1), ho, ho,
        out=o if args.residual else None, ch_scale=sc, ch_shift=sh, residual=res, relu=True,
        codes_a=ca, quant_a=(0.05, 9, 3), config=13, kc_steps=layer.kc_steps_nonneg,
        kc_chunk=getattr(layer, "kc_chunk_nonneg", -1))
    lib = tq_native.lib()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    assert lib.tq_ring_trace_clear() == 0
    fn()
    torch.cuda.synchronize()
    buf = np.zeros((1024, 8, 4), dtype=np.uint64)
    lib.tq_ring_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert lib.tq_ring_trace_read(buf.ctypes.data, buf.size) == 0
    used = buf[:, :, 0] > 0
    t = buf.astype(np.int64)
    base = t[used][:, 0].min() if used.any() else 0
    ph = ["first barrier", "K loop", "epilogue"]
    print("layer %d (%s): %d workgroups, tiles per workgroup %s" % (
        args.layer, "residual" if args.residual else "codes", int(used.any(axis=1).sum()),
        np.bincount(used.sum(axis=1))[1:].tolist()))
    for j in range(8):
        m = used[:, j]
        if not m.any():
            break
        d = (t[m, j, 1:] - t[m, j, :-1]) / 100.0  # us per phase
        st = (t[m, j, 0] - base) / 100.0
        print("tile %d: n %3d  start %6.1f us  " % (j, int(m.sum()), st.mean()) + "  ".join(
            "%s %5.2f (max %5.2f)" % (ph[i], d[:, i].mean(), d[:, i].max()) for i in range(3)))
    end = (t[used][:, 3].max() - base) / 100.0
    print("span %.1f us (first start to last epilogue issue)" % end)


if __name__ == "__main__":
    main()
