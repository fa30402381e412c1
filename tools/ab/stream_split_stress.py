"""Stress of forward() vs forward_streams() bit-identity (tests/test_gpu_fused_parity.py
test_stream_split_is_bit_identical) and of forward() against itself: on any mismatch, which
images (rows) differ.  python tools/ab/stream_split_stress.py [reps]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))
os.environ.setdefault("TQ_CONV_ENGINE", "mfma")
import bench  # noqa: E402
import tq_fuse  # noqa: E402
import util  # noqa: E402

dev = torch.device("cuda:0")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
_, q, _ = bench.build_model(dev, 256, 0)
x, _ = util.SyntheticImageNet(512, 256, seed=0, device=dev).batch(0)
x = x.contiguous(memory_format=torch.channels_last)
t0 = time.time()
with torch.no_grad():
    f = tq_fuse.FusedResNet(q)
    ref = f(x)
    torch.cuda.synchronize()
    total = {}
    for r in range(reps):
        for s2 in (1, 2, 4):
            if s2 == 1:
                got = f(x)
            else:
                streams = [torch.cuda.Stream(dev) for _ in range(s2)]
                got = f.forward_streams(x, streams)
            torch.cuda.synchronize()
            rows = torch.nonzero((ref != got).any(dim=1)).flatten().tolist()
            total[s2] = total.get(s2, 0) + (1 if rows else 0)
            if rows:
                print("rep %d, %d streams: %d rows differ: %s" % (r, s2, len(rows), rows[:16]),
                      flush=True)
        if r % 10 == 9:
            print("rep %d done (%.0f s), mismatching calls so far %s" % (r, time.time() - t0,
                                                                       total), flush=True)
print("mismatching calls of %d per mode: %s" % (reps, total))
