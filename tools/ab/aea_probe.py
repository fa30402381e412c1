"""Time tq_act_encode_act (gate, no act: EfficientNet-b0's project-conv input pass) on the
dw output shapes of EfficientNet-b0 at a 128-image chunk; select a build with TQ_LIB_PATH.
    python tools/ab/aea_probe.py [--iters 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "term-quantization_amd"))
import tq_native  # noqa: E402

SHAPES = [(32, 112), (96, 56), (144, 56), (144, 28), (240, 28), (240, 14), (480, 14),
          (672, 14), (672, 7), (1152, 7)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--n", type=int, default=128)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    total_us, total_b = 0.0, 0
    digest = 0
    for c, h in SHAPES:
        x = torch.randn(a.n, c, h, h, generator=g).to(dev).contiguous(
            memory_format=torch.channels_last)
        gate = torch.rand(a.n, c, generator=g).to(dev)
        cp = (c + 7) // 8 * 8
        codes = torch.empty(a.n, h, h, cp, dtype=torch.int16, device=dev)
        tq_native.act_encode_act(x, 0.05, 8, 3, codes, gate=gate)
        torch.cuda.synchronize()
        digest = (digest * 31 + int(codes.to(torch.int64).sum().item())) % (1 << 61)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            tq_native.act_encode_act(x, 0.05, 8, 3, codes, gate=gate)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        b = x.numel() * 4 + codes.numel() * 2
        total_us += us
        total_b += b
        print("aea C=%4d H=%3d  %7.1f us  %6.0f GB/s" % (c, h, us, b / us / 1e3))
    print("aea total %.1f us  %.0f GB/s  codes digest %d" % (total_us, total_b / total_us / 1e3,
                                                             digest))


if __name__ == "__main__":
    main()
