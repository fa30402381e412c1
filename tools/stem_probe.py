"""Run the fused stem kernel (tq_stem_conv_pool_encode) on a ResNet-18 bench batch (timing /
PMC collection).   python tools/stem_probe.py [--iters 20] [--batch 256]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import tq_native  # noqa: E402
import tq_ops  # noqa: E402
from microbench import time_fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    n = args.batch
    x = torch.randn(n, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
    w = torch.randn(64, 3, 7, 7, device=dev) * 0.05
    ws = tq_ops.pack_stem_weight(w)
    sc = torch.rand(64, device=dev) + 0.5
    sh = torch.randn(64, device=dev) * 0.1
    out = torch.empty((n, 64, 56, 56), device=dev).contiguous(memory_format=torch.channels_last)
    codes = torch.empty((n, 56, 56, 64), dtype=torch.float16, device=dev)
    fn = lambda: tq_native.stem_conv_pool_encode(x, ws, sc, sh, out, codes_a=codes,
                                                 quant_a=(0.05, 9, 3))
    t = time_fn(fn, args.iters)
    mac = n * 64 * 112 * 112 * 147
    print("stem: %.1f us  %.1f TFLOP/s fp32-equivalent" % (t * 1e6, 2 * mac / t / 1e12))


if __name__ == "__main__":
    main()
