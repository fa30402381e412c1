"""Per-launch times of the fused ResNet-18 TQ executor (the bench workload), in launch order.

    python tools/layer_times.py [--steps 5] [--batch 256]

HIP events around every TQ kernel on its launch stream; prints the average duration of each
launch position over the steps, with its layer shape.  With TQ_LIB_PATH pointing at an
ablation build (tools/ab/ablate.sh) it shows what each part of a kernel costs (timing only)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))

import bench  # noqa: E402
import tq_fuse  # noqa: E402
import tq_ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    os.environ.setdefault("TQ_CONV_ENGINE", "mfma")
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = True
    _, qmodel, _ = bench.build_model(dev, args.batch, 0)
    runner = tq_fuse.FusedResNet(qmodel)
    x = torch.randn(args.batch, 3, 224, 224, device=dev).contiguous(
        memory_format=torch.channels_last)
    seq = []

    def hook(name, work, fn, nbytes=0):
        s = torch.cuda.current_stream()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(s)
        r = fn()
        b.record(s)
        seq.append((name, work, a, b))
        return r

    with torch.no_grad():
        for _ in range(2):
            runner(x)
        torch.cuda.synchronize()
        tq_ops.set_kernel_hook(hook)
        for _ in range(args.steps):
            runner(x)
        torch.cuda.synchronize()
        tq_ops.set_kernel_hook(None)
    per = len(seq) // args.steps
    tot = 0.0
    for i in range(per):
        ts = [seq[s * per + i][2].elapsed_time(seq[s * per + i][3]) * 1e3
              for s in range(args.steps)]
        t = sum(ts) / len(ts)
        name, work = seq[i][0], seq[i][1]
        tot += t
        rate = ("%7.1f TMAC/s" % (work / t / 1e6)) if name.startswith("conv") else \
            ("%7.0f GB/s" % (work / t / 1e3))
        print("%2d %-18s %8.1f us  %s" % (i, name, t, rate))
    print("total %.1f us" % tot)


if __name__ == "__main__":
    main()
