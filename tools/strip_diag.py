"""Where do the strip engine (config 11) and the direct engine (config 10) disagree?
Prints, per shape, the mismatching (image, row % 4, column block of 32 tile pixels, channel
block) pattern of the next-layer codes.  Diagnostic only."""
import os
import sys

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))
import tq_native  # noqa: E402
import tr_layer  # noqa: E402

DEV = "cuda:0"
os.environ["TQ_CONV_ENGINE"] = "mfma"
for n, h, w in [(3, 56, 56), (5, 13, 24), (2, 9, 8)]:
    torch.manual_seed(n * 100 + h)
    conv = nn.Conv2d(64, 64, 3, 1, 1, bias=False)
    if os.environ.get("KAIMING"):
        nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
    lay = tr_layer.TRConv2dLayer(conv.to(DEV), 9, 3, 9, 8, 12)
    x = torch.relu(torch.randn(n, 64, h, w, device=DEV)).contiguous(
        memory_format=torch.channels_last)
    codes = torch.empty((n, h, w, 64), dtype=torch.float16, device=DEV)
    tq_native.act_encode(x, True, 0.02, 9, 3, codes)
    sc = torch.rand(64, dtype=torch.float64, device=DEV) * 1e-4
    sh = torch.randn(64, dtype=torch.float64, device=DEV) * 0.1
    outs = []
    for cfg in (10, 11):
        ca = torch.full((n, h, w, 64), float("nan"), dtype=torch.float16, device=DEV)
        tq_native.conv2d_termpair_fused(codes, lay.w_codes, 64, 3, 3, (1, 1), (1, 1), (1, 1),
                                        h, w, ch_scale=sc, ch_shift=sh, relu=True, codes_a=ca,
                                        quant_a=(0.05, 9, 3), config=cfg,
                                        kc_steps=lay.kc_steps_nonneg)
        outs.append(ca.view(torch.int16).cpu())
    bad = (outs[0] != outs[1])
    print((n, h, w), "mismatches", int(bad.sum()), "of", bad.numel(), flush=True)
    if bad.any():
        idx = bad.nonzero()
        img, row, col, ch = idx.unbind(1)
        tpix = (row % 4) * w + col
        pats = sorted(set(zip(img.tolist(), (row // 4).tolist(), (tpix // 32).tolist(),
                              (ch // 32).tolist())))
        print("  (img, tile, block, chblock):", pats[:40], len(pats), flush=True)
        print("  zero in strip:", int((outs[1][bad] == 0).sum()), "nan:",
              int((outs[1][bad] == outs[1].new_tensor(-512)).sum()), flush=True)
