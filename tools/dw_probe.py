"""Run one depthwise term-pair layer repeatedly (fused epilogue: BN + ReLU6 + next codes), for
PMC collection / A-B timing.  python tools/dw_probe.py --c 144 --hw 56 --stride 1 --iters 50"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import tq_native  # noqa: E402
import tr_layer  # noqa: E402
from microbench import time_fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c", type=int, default=144)
    ap.add_argument("--hw", type=int, default=56)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    c, h, s = args.c, args.hw, args.stride
    conv = torch.nn.Conv2d(c, c, 3, s, 1, groups=c, bias=False)
    layer = tr_layer.TRConv2dLayer(conv.to(dev), 9, 3, 16, 1, 16)
    cp = layer.act_channels
    x = torch.relu(torch.randn(args.batch, c, h, h, device=dev)).contiguous(
        memory_format=torch.channels_last)
    codes = torch.zeros((args.batch, h, h, cp), dtype=torch.int16, device=dev)
    tq_native.act_encode(x, True, 0.02, 9, 3, codes)
    ho = (h + 2 - 3) // s + 1
    sc = torch.rand(c, dtype=torch.float64, device=dev) * 1e-5
    sh = torch.randn(c, dtype=torch.float64, device=dev) * 0.1
    nc = torch.empty((args.batch, ho, ho, cp), dtype=torch.int16, device=dev)
    fn = lambda: tq_native.dwconv2d_termpair_fused(codes, c, layer.w_codes, 3, 3, (s, s), (1, 1),  # noqa
                                                   (1, 1), ho, ho, sc, sh, 6, next_codes=nc,
                                                   quant=(0.03, 9, 3))
    t = time_fn(fn, args.iters)
    nbytes = codes.numel() * 2 + nc.numel() * 2
    print("dw c=%d hw=%d s=%d: %.1f us  %.0f GB/s (codes in + codes out)" % (
        c, h, s, t * 1e6, nbytes / t / 1e9))


if __name__ == "__main__":
    main()
