"""Library reference points for the term-pair convs' MFMA efficiency: hipBLASLt fp16 GEMMs of
each ResNet-18 TQ conv's implicit-GEMM shape (M = Cout, N = batch*Ho*Wo, K = Cin*KH*KW) and
MIOpen's fp16 channels-last conv of the same layer, timed with events (no epilogue, no exact
int32 sums -- an upper bound for what a plain library kernel reaches on these shapes).

    python tools/gemm_ref.py [--layers 2 6 11 16] [--batch 256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
from microbench import RESNET18_TR, time_fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, nargs="*", default=[2, 6, 11, 16])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = True
    for li in args.layers:
        cin, cout, k, s, hin = RESNET18_TR[li - 1]
        ho = (hin + 2 * (k // 2) - k) // s + 1
        M, N, K = cout, args.batch * ho * ho, cin * k * k
        a = torch.randn(M, K, device=dev, dtype=torch.float16)
        b = torch.randn(K, N, device=dev, dtype=torch.float16)
        t = time_fn(lambda: torch.mm(a, b), args.iters)
        x = torch.randn(args.batch, cin, hin, hin, device=dev, dtype=torch.float16).to(
            memory_format=torch.channels_last)
        conv = torch.nn.Conv2d(cin, cout, k, s, k // 2, bias=False).to(dev).half().to(
            memory_format=torch.channels_last)
        with torch.no_grad():
            tc = time_fn(lambda: conv(x), args.iters)
        mac = M * N * K
        print("layer %2d M %d N %d K %d: gemm %.1f us (%.0f TFLOP/s, %.3f of 2.5 PF)  "
              "miopen conv %.1f us (%.3f)" % (li, M, N, K, t * 1e6, 2 * mac / t / 1e12,
                                              2 * mac / t / 2.5e15, tc * 1e6,
                                              2 * mac / tc / 2.5e15), flush=True)


if __name__ == "__main__":
    main()
