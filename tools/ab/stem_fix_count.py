"""Fused-stem exact fix-up at the bench config: how many outputs the stem lists for the
fix-up (the workspace's per-workgroup counts) and the stem's time with / without it, on
bench batch 0 (256 images, or its first N).  python tools/ab/stem_fix_count.py [N ...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))
os.environ.setdefault("TQ_CONV_ENGINE", "mfma")
import bench  # noqa: E402
import tq_fuse  # noqa: E402
import tq_native  # noqa: E402
import util  # noqa: E402

dev = torch.device("cuda:0")
_, q, _ = bench.build_model(dev, 256, 0)
x, _ = util.SyntheticImageNet(512, 256, seed=0, device=dev).batch(0)
x_all = x.contiguous(memory_format=torch.channels_last)
f = tq_fuse.FusedResNet(q, stem="exact")
for nimg in [int(v) for v in sys.argv[1:]] or [256]:
    x = x_all[:nimg].contiguous(memory_format=torch.channels_last)
    print("== %d images" % nimg)
    first = f.blocks[0]
    n, _, h, w = x.shape
    out = torch.empty((n, 64, h // 4, w // 4), device=dev).contiguous(memory_format=torch.channels_last)
    codes = torch.empty((n, h // 4, w // 4, first.conv1.cp_in), dtype=first.conv1.code_dtype,
                        device=dev)
    ws = tq_native.stem_workspace(n, h, w, dev)


    def run(exact):
        tq_native.stem_conv_pool_encode(x, f.stem_w, f.stem_scale, f.stem_shift, out, codes_a=codes,
                                        quant_a=first.conv1.quant, exact=f.stem_exact if exact else None,
                                        workspace=ws)


    run(True)
    torch.cuda.synchronize()
    cnt = ws[:4096].view(torch.int32)[:256].cpu()
    print("listed entries: total %d, per workgroup max %d mean %.1f (of %d pooled outputs)"
          % (int(cnt.sum()), int(cnt.max()), float(cnt.float().mean()), out.numel()))
    for exact in (False, True, False, True):
        for _ in range(3):
            run(exact)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run(exact)
        e1.record()
        torch.cuda.synchronize()
        print("exact=%s: %.1f us per stem call" % (exact, e0.elapsed_time(e1) / 20 * 1e3))
