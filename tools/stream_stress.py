"""Stress the fused ResNet-18 executor's chunk-stream split (forward_streams, bench.py --streams)
for bit-identity with forward() at the bench batch: 25 calls each at 2, 3 and 4 streams; prints
the logit rows of any mismatch.  python tools/stream_stress.py"""
import os, sys, torch
sys.path.insert(0, '/root/repo/term-quantization_amd'); sys.path.insert(0, '/root/repo')
os.environ.setdefault("TQ_CONV_ENGINE", "mfma")
import bench, tq_fuse
dev = torch.device('cuda:0')
_, q, _ = bench.build_model(dev, 256, 0)
x = torch.randn(256, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
f = tq_fuse.FusedResNet(q)
with torch.no_grad():
    ref = f(x)
    bad = 0
    for n in (2, 3, 4):
        streams = [torch.cuda.Stream(dev) for _ in range(n)]
        for it in range(25):
            got = f.forward_streams(x, streams)
            torch.cuda.synchronize()
            if not torch.equal(ref, got):
                bad += 1
                d = (ref - got).abs()
                rows = (d.amax(1) > 0).nonzero().flatten().tolist()
                print("MISMATCH streams", n, "iter", it, "rows", rows[:20], "max", d.max().item(), flush=True)
        r2 = f(x); torch.cuda.synchronize()
        print("streams", n, "done; forward repeat equal:", torch.equal(ref, r2), flush=True)
    print("total mismatches", bad)
