"""Reference timings of MIOpen's own fp16 / bf16 convs for the ResNet-18 TR conv shapes
(channels_last, batch 256): what a vendor dense conv of the same GEMM shape costs here.
Timing context only -- the product never calls these."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from microbench import RESNET18_TR, time_fn  # noqa: E402


def main():
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda:0")
    seen = set()
    for dt in (torch.float16,):
        total = 0.0
        for i, (cin, cout, k, s, hin) in enumerate(RESNET18_TR):
            key = (cin, cout, k, s, hin)
            x = torch.randn(256, cin, hin, hin, device=dev, dtype=dt).to(
                memory_format=torch.channels_last)
            w = torch.randn(cout, cin, k, k, device=dev, dtype=dt).to(
                memory_format=torch.channels_last)
            fn = lambda: F.conv2d(x, w, None, s, k // 2)
            t = time_fn(fn, 10)
            ho = (hin + 2 * (k // 2) - k) // s + 1
            mac = 256 * cout * ho * ho * cin * k * k
            total += t
            if key not in seen:
                print("%s conv%02d %s: %.1f us  %.1f TFLOP/s" % (dt, i + 1, key, t * 1e6,
                                                                  2 * mac / t / 1e12))
                seen.add(key)
        print("%s total %.2f ms" % (dt, total * 1e3))


if __name__ == "__main__":
    main()
