"""forward() vs forward_streams() bit-identity on the bench batch, repeated, plus the stem's
own codes on 256 images vs two 128-image halves (exact and split stems).
python tools/ab/stream_split_diag.py [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))
os.environ.setdefault("TQ_CONV_ENGINE", "mfma")
import bench  # noqa: E402
import tq_fuse  # noqa: E402
import util  # noqa: E402

dev = torch.device("cuda:0")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
_, q, _ = bench.build_model(dev, 256, 0)
x, _ = util.SyntheticImageNet(512, 256, seed=0, device=dev).batch(0)
x = x.contiguous(memory_format=torch.channels_last)
with torch.no_grad():
    for stem in ("exact", "fused"):
        f = tq_fuse.FusedResNet(q, stem=stem)
        first = f.blocks[0]
        _, c_all, _ = f._stem_fused(x, first)
        parts = [f._stem_fused(xc.contiguous(memory_format=torch.channels_last), first)[1]
                 for xc in x.chunk(2)]
        torch.cuda.synchronize()
        c_half = torch.cat(parts)
        print("%s stem: codes 256 vs 2x128 differ in %d of %d" % (
            stem, int((c_all != c_half).sum()), c_all.numel()))
        for s2 in (2, 4):
            streams = [torch.cuda.Stream(dev) for _ in range(s2)]
            ref = f(x)
            bad = []
            for _ in range(reps):
                got = f.forward_streams(x, streams)
                torch.cuda.synchronize()
                bad.append(int((ref != got).any(dim=1).sum()))
            ref2 = f(x)
            torch.cuda.synchronize()
            print("%s stem, %d streams: rows differing per rep %s; forward() repeat equal: %s"
                  % (stem, s2, bad, bool(torch.equal(ref, ref2))))
