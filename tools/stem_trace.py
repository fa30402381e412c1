"""Per-tile phase timing of one fused-stem launch at the bench batch, from the timing-only build
`bash tools/ab/variant1.sh strace tq_stem_conv "-DSTEM_TRACE=1"` (wave 0's s_memrealtime stamps per
tile: loop top, barrier A passed (tile max known), barrier B passed (rows committed), tile done;
select it with TQ_LIB_PATH).   python tools/stem_trace.py"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))

import tq_native  # noqa: E402
import tq_ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    n = 256
    x = torch.randn(n, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
    ws = tq_ops.pack_stem_weight(torch.randn(64, 3, 7, 7, device=dev) * 0.05)
    sc = torch.rand(64, device=dev) + 0.5
    sh = torch.randn(64, device=dev) * 0.1
    out = torch.empty((n, 64, 56, 56), device=dev).contiguous(memory_format=torch.channels_last)
    codes = torch.empty((n, 56, 56, 64), dtype=torch.float16, device=dev)
    fn = lambda: tq_native.stem_conv_pool_encode(x, ws, sc, sh, out, codes_a=codes,  # noqa: E731
                                                 quant_a=(0.05, 9, 3))
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    fn()
    torch.cuda.synchronize()
    buf = np.zeros((1024, 16, 4), dtype=np.uint64)
    lib = tq_native.lib()
    lib.tq_stem_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert lib.tq_stem_trace_read(buf.ctypes.data, buf.size) == 0
    t = buf.astype(np.int64)
    used = t[:, :, 0] > 0
    base = t[used][:, 0].min()
    d = (t[:, :, 1:] - t[:, :, :-1]) / 100.0
    names = ["top -> barrier A (max / wait)", "A -> B (commit rows)", "B -> tile done (convs, pool, stores)"]
    for i, nm in enumerate(names):
        v = d[:, :, i][used]
        print("%-40s mean %6.2f us  max %6.2f  total per workgroup %7.1f us" % (
            nm, v.mean(), v.max(), v.sum() / used.any(axis=1).sum()))
    wv = np.zeros((1024, 16, 8, 3), dtype=np.uint64)
    lib.tq_stem_trace_waves_read.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert lib.tq_stem_trace_waves_read(wv.ctypes.data, wv.size) == 0
    wa = wv.astype(np.int64)[used]  # [tiles, 8 waves, 3 stamps]
    b = t[used][:, 2][:, None]      # barrier B passed (wave 0)
    for k, nm in enumerate(["after the prefetch issue", "after pass 0", "tile done"]):
        print("per wave, %-26s (us after barrier B): %s" % (
            nm, np.round(((wa[:, :, k] - b) / 100.0).mean(0), 2).tolist()))
    print("tiles per workgroup %s, span %.1f us" % (np.bincount(used.sum(axis=1))[1:].tolist(),
                                                   (t[used][:, 3].max() - base) / 100.0))


if __name__ == "__main__":
    main()
