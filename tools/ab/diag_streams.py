"""Stress check: forward() vs forward_streams() logits of the fused ResNet-18 executor on the
bench batch, repeated, with the c64 engine on and off (TQ_C64).  Prints mismatching rows."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))
os.environ["TQ_CONV_ENGINE"] = "mfma"
import bench  # noqa: E402
import tq_fuse  # noqa: E402
import util  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
_, qmodel, _ = bench.build_model(dev, 256, 0)
x, _ = util.SyntheticImageNet(512, 256, seed=0, device=dev).batch(0)
x = x.contiguous(memory_format=torch.channels_last)
fused = tq_fuse.FusedResNet(qmodel, stem="fused")  # (the r05 stem: no fix-up)
for flag in ("1", "0"):
    os.environ["TQ_C64"] = flag
    with torch.no_grad():
        ref = fused(x)
        for ns in (2, 4):
            streams = [torch.cuda.Stream(dev) for _ in range(ns)]
            nbad = 0
            for rep in range(reps):
                got = fused.forward_streams(x, streams)
                again = fused(x)
                torch.cuda.synchronize()
                d = (got - ref).abs()
                bad = (d > 0).any(dim=1).nonzero().flatten().tolist()
                d2 = (again - ref).abs()
                bad2 = (d2 > 0).any(dim=1).nonzero().flatten().tolist()
                if bad or bad2:
                    nbad += 1
                    print("TQ_C64=%s streams %d rep %d: streams rows %s (max %.3g); forward rows %s"
                          % (flag, ns, rep, bad[:10], d.max().item(), bad2[:10]), flush=True)
            print("TQ_C64=%s streams %d: %d of %d reps differ" % (flag, ns, nbad, reps),
                  flush=True)
