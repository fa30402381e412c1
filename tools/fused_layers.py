"""Per-launch timings of one fused MobileNet-V2 / EfficientNet-b0 forward (tq_ops kernel
hook, HIP events around each TQ kernel): name, algorithmic bytes, microseconds, GB/s.

    python tools/fused_layers.py --arch mobilenet_v2
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))
import cnn_models  # noqa: E402
import tq_fuse  # noqa: E402
import tq_ops  # noqa: E402
import tr_layer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="mobilenet_v2")
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = getattr(cnn_models, args.arch)(pretrained=False).to(dev).eval()
    settings = cnn_models.static_conv_layer_settings(model, 9, 8, 12)
    q = cnn_models.convert_model(model, settings, 9, 3).to(memory_format=torch.channels_last)
    x = torch.randn(args.batch, 3, 224, 224, device=dev).contiguous(
        memory_format=torch.channels_last)
    rec = []

    def hook(name, work, fn, nbytes=0):
        s = torch.cuda.current_stream()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(s)
        r = fn()
        b.record(s)
        rec.append((name, work, nbytes, a, b))
        return r

    with torch.no_grad():
        q(x)
        tr_layer.set_tr_tracking(q, False)
        ex = (tq_fuse.FusedMobileNetV2 if args.arch == "mobilenet_v2" else
              tq_fuse.FusedEfficientNet)(q)
        for _ in range(3):
            ex(x)
        torch.cuda.synchronize()
        tq_ops.set_kernel_hook(hook)
        try:
            ex(x)
            torch.cuda.synchronize()
        finally:
            tq_ops.set_kernel_hook(None)
    tot = 0.0
    for i, (name, work, nbytes, a, b) in enumerate(rec):
        us = a.elapsed_time(b) * 1e3
        tot += us
        print("%3d %-24s bytes %10.1f MB  %8.1f us  %7.0f GB/s  work %.3g" % (
            i, name, nbytes / 1e6, us, nbytes / us / 1e3 if us else 0, work))
    print("sum of launches %.1f us" % tot)


if __name__ == "__main__":
    main()
