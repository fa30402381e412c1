"""Adversarial GPU checks of the MFMA engine's exactness windows and of the epilogue's code
padding.

* Weights whose window sums sit just under 2^24 / 2^db, with activation codes saturated at
  maxv, so that a window one K-step wider than the host computed would carry an odd partial
  sum above 2^24 (not an fp32 value).  Every MFMA tile config, run with the wider
  non-negative windows (tq_ops.mfma_flush_steps / mfma_flush_chunk(nonneg=True)), must give
  the VALU engine's exact int32 sums bit for bit.
* Cout % 8 == 4: the fused epilogue must zero the pad channels of the codes it emits, so a
  consumer never multiplies stale fp16 bits (Inf/NaN) by its zero pad weights."""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import oracle
import tq_native
import tq_ops
import tr_layer

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

SAT, ONE = 30, 1   # channels 0..29 at code 511, channel 30 at code 1, the rest 0


def _weights(cin, cout):
    """Codes +255 on channels < 32, -255 on channels >= 32 (rows < cout - 1); the last row
    holds the single 256 that sets w_sf = max|w| / 2^8 so that 255 is a code."""
    w = torch.zeros(cout, cin, 3, 3)
    w[:cout - 1, :32] = 255.0
    w[:cout - 1, 32:] = -255.0
    w[cout - 1, 0, 0, 0] = 256.0
    return w * 1e-3


def _layer(cin, cout, stride, engine, monkeypatch):
    monkeypatch.setenv("TQ_CONV_ENGINE", engine)
    conv = nn.Conv2d(cin, cout, 3, stride, 0, bias=False)
    with torch.no_grad():
        conv.weight.copy_(_weights(cin, cout))
    lay = tr_layer.TRConv2dLayer(conv.to(DEV), 9, 3, 9, 1, 9)  # g=1, k=9 keeps every term
    assert lay.engine == engine
    return lay


def _act(n, cin, hw):
    sf = 0.01
    x = torch.zeros(n, cin, hw, hw)
    x[:, :SAT] = 600 * sf       # saturates: q = 511 = 512 - 1 (two terms)
    x[:, SAT:SAT + ONE] = sf    # q = 1
    return x.to(DEV).contiguous(memory_format=torch.channels_last), sf


@pytest.mark.parametrize("cout,stride,hw", [(64, 1, 12), (256, 1, 16), (256, 2, 17),
                                            (128, 2, 15)])
def test_nonneg_windows_at_the_bound(cout, stride, hw, monkeypatch):
    cin, n = 64, 3
    lay_m = _layer(cin, cout, stride, "mfma", monkeypatch)
    codes_w = lay_m.w_codes[:cout - 1, :9 * 64].float()
    assert bool((codes_w.abs() == 255).all())
    # general window: 2^9 * 64 * 255 per K-step -> 2 steps; non-negative: 2^9 * 32 * 255 -> 4
    assert lay_m.kc_steps == 2 and lay_m.kc_steps_nonneg == 4
    assert lay_m.kc_chunk in (2, -1) and lay_m.kc_chunk_nonneg == 4
    x, sf = _act(n, cin, hw)
    ho = (hw - 3) // stride + 1
    # exact per-row sums: 9 taps x (30 * 255 * 511 + 255) (odd per step; 5 steps > 2^24)
    per_step = SAT * 255 * 511 + 255
    assert per_step * 4 <= 2**24 < per_step * 5 and per_step % 2 == 1
    total = 9 * per_step
    sc = torch.ones(cout, dtype=torch.float64, device=DEV)
    sh = torch.full((cout,), -float(total), dtype=torch.float64, device=DEV)
    sh[cout - 1] = -256.0 * 511
    outs = []
    cm = torch.empty((n, hw, hw, 64), dtype=torch.float16, device=DEV)
    tq_native.act_encode(x, True, sf, 9, 3, cm)
    for cfg in range(0, tq_native.lib().tq_conv2d_mfma_num_configs() + 1):
        o = torch.full((n, cout, ho, ho), float("nan"), device=DEV).contiguous(
            memory_format=torch.channels_last)
        tq_native.conv2d_termpair_fused(cm, lay_m.w_codes, cout, 3, 3, (stride, stride),
                                        (0, 0), (1, 1), ho, ho, out=o, ch_scale=sc, ch_shift=sh,
                                        config=cfg, kc_steps=lay_m.kc_steps_nonneg,
                                        kc_chunk=lay_m.kc_chunk_nonneg)
        outs.append(o.cpu())
    lay_v = _layer(cin, cout, stride, "valu", monkeypatch)
    ci = torch.empty((n, hw, hw, 64), dtype=torch.int16, device=DEV)
    tq_native.act_encode(x, True, sf, 9, 3, ci)
    o = torch.full((n, cout, ho, ho), float("nan"), device=DEV).contiguous(
        memory_format=torch.channels_last)
    tq_native.conv2d_termpair_fused(ci, lay_v.w_codes, cout, 3, 3, (stride, stride), (0, 0),
                                    (1, 1), ho, ho, out=o, ch_scale=sc, ch_shift=sh)
    ref = o.cpu()
    # y = acc - expected: exactly 0 everywhere when every partial sum was exact
    assert torch.equal(ref, torch.zeros_like(ref))
    for i, got in enumerate(outs):
        assert torch.equal(got, ref), "config %d" % i


@pytest.mark.parametrize("engine", ["mfma", "valu"])
def test_epilogue_zeroes_code_padding(engine, monkeypatch):
    """Cout = 12: codes_a has Cp = 16, the epilogue writes channels 12..15 as zero codes even
    into a buffer prefilled with NaN bits; the consumer then matches the fp64 reference."""
    import tq_fuse
    monkeypatch.setenv("TQ_CONV_ENGINE", engine)
    torch.manual_seed(21)
    c1 = nn.Conv2d(16, 12, 3, 1, 1, bias=False)
    c2 = nn.Conv2d(12, 20, 3, 1, 1, bias=True)
    a = tr_layer.TRConv2dLayer(c1.to(DEV), 9, 3, 9, 4, 6)
    b = tr_layer.TRConv2dLayer(c2.to(DEV), 9, 3, 9, 4, 6)
    for lay, sf in ((a, 0.03), (b, 0.05)):
        lay.input_quant.tracking = False
        lay.input_quant.sf = sf
    ca, cb = tq_fuse._Conv(a, None), tq_fuse._Conv(b, None)
    x = torch.relu(torch.randn(2, 16, 9, 9, device=DEV)).contiguous(
        memory_format=torch.channels_last)
    codes = torch.empty((2, 9, 9, 16), dtype=ca.code_dtype, device=DEV)
    tq_native.act_encode(x, True, 0.03, 9, 3, codes)
    mid = torch.empty((2, 9, 9, 16), dtype=cb.code_dtype, device=DEV)
    mid.view(torch.int16).fill_(0x7E00 if engine == "mfma" else -1)  # NaN fp16 / junk
    y1 = torch.empty((2, 12, 9, 9), device=DEV).contiguous(memory_format=torch.channels_last)
    ws = tq_native.conv2d_workspace(2 * 81, 12, DEV)
    tq_native.conv2d_termpair_fused(codes, a.w_codes, 12, 3, 3, (1, 1), (1, 1), (1, 1), 9, 9,
                                    out=y1, ch_scale=ca.scale, ch_shift=ca.shift, relu=True,
                                    codes_a=mid, quant_a=cb.quant, workspace=ws,
                                    kc_steps=ca.kc_steps, kc_chunk=ca.kc_chunk)
    assert not mid[..., 12:].view(torch.int16).any()
    y2 = torch.empty((2, 20, 9, 9), device=DEV).contiguous(memory_format=torch.channels_last)
    ws2 = tq_native.conv2d_workspace(2 * 81, 20, DEV)
    tq_native.conv2d_termpair_fused(mid, b.w_codes, 20, 3, 3, (1, 1), (1, 1), (1, 1), 9, 9,
                                    out=y2, ch_scale=cb.scale, ch_shift=cb.shift,
                                    workspace=ws2, kc_steps=cb.kc_steps, kc_chunk=cb.kc_chunk)
    yq = oracle.tr(y1.contiguous().cpu().numpy().reshape(1, -1, 1, 1), 0.05, 9, 1, 3)
    xq = torch.from_numpy(yq).view(y1.shape).double()
    wq = b.conv.weight.detach().double().cpu()
    ref = F.conv2d(xq, wq, b.conv.bias.detach().double().cpu(), 1, 1)
    mag = F.conv2d(xq.abs(), wq.abs(), None, 1, 1)
    got = y2.double().cpu()
    assert bool(torch.isfinite(got).all())
    assert bool(((got - ref).abs() <= 1e-5 * torch.maximum(ref.abs(), mag) + 1e-30).all())
    exp_codes = np.rint(yq.reshape(y1.shape) / np.float32(0.05)).astype(np.int64)
    assert torch.equal(mid[..., :12].cpu().long().permute(0, 3, 1, 2),
                       torch.from_numpy(exp_codes))


@pytest.mark.parametrize("engine", ["mfma", "valu"])
@pytest.mark.parametrize("shift", [0.0, 1e-7, -1e-7, 3.3e-6])
def test_epilogue_codes_at_rounding_midpoints(engine, shift, monkeypatch):
    """The epilogue's fast path for the next layer's codes (division-free quotient, fract
    rounding, top-bit peel) against the oracle's true division, on outputs that sit on and
    around rounding midpoints: a 1x1 conv whose weights are 256 * identity,
    scale sc, and next sf = 2 * sc * 256 / 256, so y / sf = acc / 512 * 256 / 2 = x_code / 2
    -- every odd activation code lands on q + 0.5 exactly (before the shift moves it by a
    few ulps)."""
    import tq_fuse
    monkeypatch.setenv("TQ_CONV_ENGINE", engine)
    c = 64
    conv = nn.Conv2d(c, c, 1, 1, 0, bias=False)
    with torch.no_grad():
        conv.weight.copy_(torch.eye(c).view(c, c, 1, 1) * 0.5)
    lay = tr_layer.TRConv2dLayer(conv.to(DEV), 10, 10, 9, 1, 9)
    lay.input_quant.tracking = False
    lay.input_quant.sf = 1.0
    cv = tq_fuse._Conv(lay, None)
    sc = 0.0371
    n, hw = 2, 16
    # activation codes 0..1023 (10 bits, all terms kept): x = code * sf_x
    xc = torch.arange(n * c * hw * hw, dtype=torch.float32).remainder(1024).view(n, c, hw, hw)
    x = xc.to(DEV).contiguous(memory_format=torch.channels_last)
    codes = torch.empty((n, hw, hw, c), dtype=cv.code_dtype, device=DEV)
    tq_native.act_encode(x, True, 1.0, 10, 10, codes)
    ws = tq_native.conv2d_workspace(n * hw * hw, c, DEV)
    scv = torch.full((c,), sc / 256.0, dtype=torch.float64, device=DEV)  # acc = 256 * code
    shv = torch.full((c,), shift, dtype=torch.float64, device=DEV)
    sf_next = 2.0 * sc
    y = torch.empty((n, c, hw, hw), device=DEV).contiguous(memory_format=torch.channels_last)
    ca = torch.empty((n, hw, hw, c), dtype=cv.code_dtype, device=DEV)
    tq_native.conv2d_termpair_fused(codes, lay.w_codes, c, 1, 1, (1, 1), (0, 0), (1, 1), hw, hw,
                                    out=y, ch_scale=scv, ch_shift=shv, relu=True, codes_a=ca,
                                    quant_a=(sf_next, 9, 3), workspace=ws,
                                    kc_steps=cv.kc_steps, kc_chunk=cv.kc_chunk)
    yn = y.contiguous().cpu().numpy()
    exp = np.rint(oracle.tr(yn.reshape(1, -1, 1, 1), sf_next, 9, 1, 3).reshape(yn.shape) /
                  np.float32(sf_next)).astype(np.int64)
    got = ca.cpu().long().permute(0, 3, 1, 2).numpy()
    np.testing.assert_array_equal(got, exp)
    # the inputs do straddle midpoints: y / sf within 4 ulps of a half-integer for many
    r = (yn / np.float32(sf_next)).astype(np.float32)
    near = np.abs(r - np.floor(r) - 0.5) <= 4 * np.spacing(r)
    assert near.sum() > 1000


@pytest.mark.parametrize("shape", [(3, 56, 56), (5, 13, 24), (37, 56, 56), (2, 9, 8)])
@pytest.mark.parametrize("mode", ["conv1", "conv2", "plain"])
def test_strip_engine_bit_identical(shape, mode, monkeypatch):
    """The row-strip engine (tr_conv_strip.hip, config 11: layer-1 shapes, 64 -> 64, 3x3/1)
    against the direct engine (config 10): the same exact integer sums and epilogue, so every
    fp32 output and code must be bit-identical -- with a partial last strip (H % 4 != 0),
    narrow images, batches that leave teams without tiles, NaN-prefilled outputs, and the
    epilogue shapes the executor uses (codes only / plain fp32; residual + fp32 + two code
    targets is not strip-eligible and must come back from the fallback unchanged)."""
    monkeypatch.setenv("TQ_CONV_ENGINE", "mfma")
    tq_native.sync_faults()  # start from a clean fault count
    n, h, w = shape
    torch.manual_seed(n * 100 + h)
    conv = nn.Conv2d(64, 64, 3, 1, 1, bias=False)
    nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
    lay = tr_layer.TRConv2dLayer(conv.to(DEV), 9, 3, 9, 8, 12)
    assert lay.engine == "mfma" and lay.kc_steps_nonneg == 0 and lay.kc_steps == 0
    x = torch.relu(torch.randn(n, 64, h, w, device=DEV)).contiguous(
        memory_format=torch.channels_last)
    codes = torch.empty((n, h, w, 64), dtype=torch.float16, device=DEV)
    tq_native.act_encode(x, True, 0.02, 9, 3, codes)
    sc = torch.rand(64, dtype=torch.float64, device=DEV) * 1e-4
    sh = torch.randn(64, dtype=torch.float64, device=DEV) * 0.1
    res = torch.randn(n, 64, h, w, device=DEV).contiguous(memory_format=torch.channels_last)
    outs = []
    for cfg in (10, 11):
        o = torch.full((n, 64, h, w), float("nan"), device=DEV).contiguous(
            memory_format=torch.channels_last)
        ca = torch.full((n, h, w, 64), float("nan"), dtype=torch.float16, device=DEV)
        cb = torch.full((n, h, w, 64), float("nan"), dtype=torch.float16, device=DEV)
        if mode == "plain":  # fp32 output only, no ReLU, no codes
            tq_native.conv2d_termpair_fused(codes, lay.w_codes, 64, 3, 3, (1, 1), (1, 1),
                                            (1, 1), h, w, out=o, ch_scale=sc, ch_shift=sh,
                                            config=cfg, kc_steps=lay.kc_steps)
        else:
            tq_native.conv2d_termpair_fused(
                codes, lay.w_codes, 64, 3, 3, (1, 1), (1, 1), (1, 1), h, w,
                out=o if mode == "conv2" else None, ch_scale=sc, ch_shift=sh,
                residual=res if mode == "conv2" else None, relu=True, codes_a=ca,
                quant_a=(0.05, 9, 3), codes_b=cb if mode == "conv2" else None,
                quant_b=(0.031, 9, 3) if mode == "conv2" else None, config=cfg,
                kc_steps=lay.kc_steps_nonneg)
        outs.append((o.cpu(), ca.cpu(), cb.cpu()))
    (o0, a0, b0), (o1, a1, b1) = outs
    assert tq_native.sync_faults() == 0  # no bounded team-sync wait ran out
    if mode != "conv1":
        assert not torch.isnan(o0).any()
        _same(o0.permute(0, 2, 3, 1), o1.permute(0, 2, 3, 1), "out")
    if mode != "plain":
        _same(a0.view(torch.int16), a1.view(torch.int16), "codes_a")
        if mode == "conv2":
            _same(b0.view(torch.int16), b1.view(torch.int16), "codes_b")


def _same(ref, got, what):
    """Bit equality of two NHWC tensors; on failure name where they differ (image, row,
    column, channel ranges) and whether the strip side holds zeros or NaN prefill."""
    if torch.equal(ref.view(torch.int32) if ref.dtype == torch.float32 else ref,
                   got.view(torch.int32) if got.dtype == torch.float32 else got):
        return
    bad = (ref != got) & ~(torch.isnan(ref.float()) & torch.isnan(got.float()))
    idx = bad.nonzero()
    lo, hi = idx.min(0).values.tolist(), idx.max(0).values.tolist()
    g = got[bad]
    raise AssertionError("%s: %d mismatches, n/h/w/c from %s to %s, first %s; strip side "
                         "zero %d, nan %d" % (what, int(bad.sum()), lo, hi, idx[:4].tolist(),
                                              int((g == 0).sum()),
                                              int(torch.isnan(g.float()).sum())))


@pytest.mark.parametrize("shape", [
    # cin, cout, stride, n, h, relu, residual: MobileNet-V2 / EfficientNet 1x1 shapes (expand,
    # project with a residual, swish), ResNet downsamples (stride 2), partial K / Cout tiles,
    # a pixel count that is not a multiple of the 128-pixel tile
    (16, 96, 1, 3, 17, 6, False), (32, 16, 1, 2, 23, 0, False), (96, 24, 1, 2, 14, 0, True),
    (24, 144, 1, 2, 9, "swish", False), (64, 128, 2, 2, 14, 0, False),
    (128, 256, 2, 1, 10, 0, False), (160, 960, 1, 1, 7, 6, False), (40, 20, 1, 3, 5, 1, True),
])
def test_pointwise_engine_bit_identical(shape, monkeypatch):
    """The persistent pointwise engine (tr_conv_direct.hip conv2d_tp_pw_kernel: 1x1 convs with
    <= 3 K-steps, weights staged once per workgroup, next tile's fragments in flight) against
    the direct engine (TQ_PW=0): the same exact sums and shared epilogue, so outputs and codes
    are bit-identical."""
    monkeypatch.setenv("TQ_CONV_ENGINE", "mfma")
    cin, cout, s, n, h, relu, resid = shape
    torch.manual_seed(cin * 7 + cout)
    conv = nn.Conv2d(cin, cout, 1, s, 0, bias=False)
    lay = tr_layer.TRConv2dLayer(conv.to(DEV), 9, 3, 9, 8, 12)
    assert lay.engine == "mfma"
    cp = lay.act_channels
    x = torch.relu(torch.randn(n, cin, h, h, device=DEV)).contiguous(
        memory_format=torch.channels_last)
    codes = torch.zeros((n, h, h, cp), dtype=torch.float16, device=DEV)
    tq_native.act_encode(x, True, 0.02, 9, 3, codes)
    ho = (h - 1) // s + 1
    sc = torch.rand(cout, dtype=torch.float64, device=DEV) * 1e-4
    sh = torch.randn(cout, dtype=torch.float64, device=DEV) * 0.1
    res = torch.randn(n, cout, ho, ho, device=DEV).contiguous(
        memory_format=torch.channels_last) if resid else None
    cpo = tq_ops.act_channels(cout)
    outs = []
    for mode in ("0", "1"):
        monkeypatch.setenv("TQ_PW", mode)
        o = torch.full((n, cout, ho, ho), float("nan"), device=DEV).contiguous(
            memory_format=torch.channels_last)
        ca = torch.full((n, ho, ho, cpo), float("nan"), dtype=torch.float16, device=DEV)
        tq_native.conv2d_termpair_fused(
            codes, lay.w_codes, cout, 1, 1, (s, s), (0, 0), (1, 1), ho, ho, out=o,
            ch_scale=sc, ch_shift=sh, residual=res, relu=relu,
            codes_a=ca if relu not in (0, "swish") else None,
            quant_a=(0.05, 9, 3) if relu not in (0, "swish") else None, kc_steps=lay.kc_steps)
        outs.append((o.cpu(), ca.cpu()))
    (o0, a0), (o1, a1) = outs
    assert not torch.isnan(o0).any()
    _same(o0.permute(0, 2, 3, 1), o1.permute(0, 2, 3, 1), "out")
    if relu not in (0, "swish"):
        _same(a0.view(torch.int16), a1.view(torch.int16), "codes_a")
