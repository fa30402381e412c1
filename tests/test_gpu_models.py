"""GPU parity of the depthwise and Linear term-pair paths and of whole converted models."""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import oracle
import tr_layer
import cnn_models
from cnn_models.efficientnet import Conv2dStaticSamePadding

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
RTOL = 1e-5


def _tr_x(x, sf, db, dt):
    return torch.from_numpy(oracle.tr(x.contiguous().cpu().numpy().reshape(1, -1, 1, 1), sf,
                                      db, 1, dt)).view(x.shape).double()


def _check(y, ref, mag):
    err = (y.double().cpu() - ref).abs()
    assert bool((err <= RTOL * torch.maximum(ref.abs(), mag) + 1e-30).all()), \
        float((err / (RTOL * torch.maximum(ref.abs(), mag) + 1e-30)).max())


@pytest.mark.parametrize("cfg", [
    # channels, k, stride, pad, hw, static-same (EfficientNet), bias
    (32, 3, 1, 1, 14, False, False), (96, 3, 2, 1, 15, False, False),
    (144, 5, 2, 0, 16, True, False), (40, 5, 1, 0, 9, True, True), (20, 3, 1, 1, 7, False, True),
])
@pytest.mark.parametrize("channels_last", [False, True])
def test_depthwise_termpair_matches_reference(cfg, channels_last):
    c, k, s, p, hw, same, bias = cfg
    torch.manual_seed(c + k)
    if same:
        conv = Conv2dStaticSamePadding(c, c, k, stride=s, groups=c, bias=bias, image_size=hw)
    else:
        conv = nn.Conv2d(c, c, k, s, p, groups=c, bias=bias)
    w = conv.weight.detach().clone()
    b = conv.bias.detach().clone() if bias else None
    layer = tr_layer.TRConv2dLayer(conv.to(DEV), 9, 3, 16, 1, 16)  # (16, 1, 16) dw settings
    assert layer.mode == "depthwise"
    layer.input_quant.tracking = False
    layer.input_quant.sf = 0.02
    x = torch.relu(torch.randn(2, c, hw, hw))
    xd = x.to(DEV)
    if channels_last:
        xd = xd.to(memory_format=torch.channels_last)
    with torch.no_grad():
        y = layer(xd)
    xq = _tr_x(x, 0.02, 9, 3)
    wq = torch.from_numpy(oracle.tr(w.numpy(), layer.w_sf, 16, 1, 16)).double()
    assert torch.equal(layer.conv.weight.detach().cpu().double(), wq)
    if same:
        xq = conv.static_padding.cpu()(xq)
    ref = F.conv2d(xq, wq, b.double() if bias else None, s, conv.padding, 1, c)
    mag = F.conv2d(xq.abs(), wq.abs(), None, s, conv.padding, 1, c)
    assert y.shape == ref.shape
    _check(y, ref, mag)


@pytest.mark.parametrize("cfg", [
    # cin, cout, k, stride, pad, hw, batch, bias, static-same
    (1152, 48, 1, 1, 0, 1, 256, True, True),    # EfficientNet-b0 squeeze-excite reduce
    (48, 1152, 1, 1, 0, 1, 256, True, True),    # ... and expand
    (20, 70, 3, 2, 1, 9, 3, False, False),      # general shape: taps, stride, padding
    (96, 24, 5, 1, 0, 12, 2, True, True),       # static "same" padding, 5x5
])
@pytest.mark.parametrize("channels_last", [False, True])
def test_wide_termpair_matches_reference(cfg, channels_last):
    """groups = 1 convs with (16, 1, 16) weights (int32 codes, int64 sums) against
    conv2d_fp64(TR(x), TR(w)) + bias, TR'd by the oracle; activations of both signs (the SE
    convs see swish outputs)."""
    cin, cout, k, s, p, hw, n, bias, same = cfg
    torch.manual_seed(cin + cout + k)
    if same:
        conv = Conv2dStaticSamePadding(cin, cout, k, stride=s, bias=bias, image_size=hw)
    else:
        conv = nn.Conv2d(cin, cout, k, s, p, bias=bias)
    w = conv.weight.detach().clone()
    b = conv.bias.detach().clone() if bias else None
    layer = tr_layer.TRConv2dLayer(conv.to(DEV), 9, 3, 16, 1, 16)
    assert layer.mode == "wide"
    layer.input_quant.tracking = False
    layer.input_quant.sf = 0.01
    x = torch.randn(n, cin, hw, hw)
    xd = x.to(DEV)
    if channels_last:
        xd = xd.to(memory_format=torch.channels_last)
    with torch.no_grad():
        y = layer(xd)
    xq = _tr_x(x, 0.01, 9, 3)
    wq = torch.from_numpy(oracle.tr(w.numpy(), layer.w_sf, 16, 1, 16)).double()
    assert torch.equal(layer.conv.weight.detach().cpu().double(), wq)
    assert float(wq.abs().max() / np.float32(layer.w_sf)) > 2**14  # codes leave int16 range
    if same:
        xq = conv.static_padding.cpu()(xq)
    ref = F.conv2d(xq, wq, b.double() if bias else None, s, conv.padding)
    mag = F.conv2d(xq.abs(), wq.abs(), None, s, conv.padding)
    assert y.shape == ref.shape
    assert y.is_contiguous(memory_format=torch.channels_last) == channels_last or hw == 1
    _check(y, ref, mag)


def test_linear_termpair_matches_reference():
    torch.manual_seed(3)
    lin = nn.Linear(650, 300)
    w = lin.weight.detach().clone()
    b = lin.bias.detach().clone()
    layer = tr_layer.TRLinearLayer(lin.to(DEV), 8, 8, 8, 8, 12, quantize_input=True)
    assert layer.termpair
    layer.input_quant.tracking = False
    layer.input_quant.sf = 0.01
    x = torch.randn(35, 10, 650)
    with torch.no_grad():
        y = layer(x.to(DEV))
    xq = _tr_x(x, 0.01, 8, 8)
    wq = torch.from_numpy(oracle.tr(w.numpy(), layer.w_sf, 8, 8, 12)).double()
    ref = xq @ wq.t() + b.double()
    mag = xq.abs() @ wq.abs().t()
    assert y.shape == (35, 10, 300)
    _check(y, ref, mag)


def test_linear_default_keeps_reference_semantics():
    torch.manual_seed(4)
    lin = nn.Linear(64, 16).to(DEV)
    layer = tr_layer.TRLinearLayer(lin, 8, 4, 8, 8, 12)
    x = torch.randn(5, 64, device=DEV)
    with torch.no_grad():
        layer(x)
        tr_layer.set_tr_tracking(nn.Sequential(layer), False)
        y = layer(x)
    # forward returns linear(x) on the unquantized input, with TR'd weights
    assert torch.allclose(y, F.linear(x, layer.linear.weight, layer.linear.bias))


@pytest.mark.parametrize("arch", ["mobilenet_v2", "efficientnet_b0"])
def test_depthwise_models_layers_match_reference_composition(arch):
    """Every converted layer of MobileNet-V2 / EfficientNet-b0, fed the same input, matches
    the reference composition conv(TR(x), TR(w)) in fp64 within 1e-5."""
    torch.manual_seed(0)
    model = getattr(cnn_models, arch)(pretrained=False).to(DEV).eval()
    settings = cnn_models.static_conv_layer_settings(model, 9, 8, 12)
    q = cnn_models.convert_model(model, settings, 9, 3)
    layers = [m for m in q.modules() if isinstance(m, tr_layer.TRConv2dLayer)]
    inputs = {}
    hooks = [m.register_forward_pre_hook(lambda m, a: inputs.__setitem__(id(m), a[0]))
             for m in layers]
    x = torch.randn(2, 3, 224, 224, device=DEV)
    with torch.no_grad():
        q(x)
    tr_layer.set_tr_tracking(q, False)
    modes = set()
    for m in layers:
        xin = inputs[id(m)]
        modes.add(m.mode)
        with torch.no_grad():
            y = m(xin)
        c = m.conv
        xq = _tr_x(xin, m.input_quant.sf, m.data_bits, m.data_terms)
        wq = c.weight.detach().cpu().double()
        pad = getattr(c, "static_padding", None)
        if pad is not None:
            xq = pad.cpu()(xq)
        b = c.bias.detach().cpu().double() if c.bias is not None else None
        ref = F.conv2d(xq, wq, b, c.stride, c.padding, c.dilation, c.groups)
        mag = F.conv2d(xq.abs(), wq.abs(), None, c.stride, c.padding, c.dilation, c.groups)
        if m.mode == "reference":
            continue  # fp32 torch conv of the fake-quantized tensors, as the reference
        _check(y, ref, mag)
    for h in hooks:
        h.remove()
    assert {"termpair", "depthwise"} <= modes
    assert "reference" not in modes  # every converted layer runs a term-pair kernel
    if arch == "efficientnet_b0":
        assert "wide" in modes  # the (16, 1, 16) squeeze-excite convs


@pytest.mark.parametrize("cfg", [
    # c, hw, stride, pad (top, left), ho/wo: plain 3x3 s1 p1, s2 p1 (odd input), MobileNet-V2
    # shapes, static-same s2 (pad 0 top/left, EfficientNet), H % 8 != 0, Cp with pad channels
    (32, 14, 1, (1, 1)), (96, 15, 2, (1, 1)), (144, 28, 2, (1, 1)), (40, 13, 1, (1, 1)),
    (24, 16, 2, (0, 0)), (20, 9, 1, (1, 1)), (960, 7, 1, (1, 1)), (32, 57, 1, (1, 1)),
    (16, 61, 2, (0, 0)),
])
@pytest.mark.parametrize("relu", [6, "swish"])
def test_dw_sliding_window_kernel_bit_identical(cfg, relu, monkeypatch):
    """The streaming 3x3 depthwise kernel (tr_dwconv.hip dwconv3_stream_kernel: R-row blocks,
    the next block's rows in flight, one- and multi-block segments) and the sliding-window
    kernel (dwconv3_slide_kernel, 4 or 8 channels per lane) against the row-blocked kernel
    (TQ_DW_SLIDE=0): the same exact int32 sums and epilogue, so the fp32 outputs and the next
    layer's codes are bit-identical, including partial row blocks and segments, odd sizes,
    stride 2 and asymmetric (static-same) padding."""
    import tq_native
    c, hw, s, (pt, pl) = cfg
    torch.manual_seed(c + hw)
    conv = nn.Conv2d(c, c, 3, s, 1, groups=c, bias=False)
    layer = tr_layer.TRConv2dLayer(conv.to(DEV), 9, 3, 16, 1, 16)
    cp = layer.act_channels
    x = torch.relu(torch.randn(3, c, hw, hw, device=DEV)).contiguous(
        memory_format=torch.channels_last)
    codes = torch.zeros((3, hw, hw, cp), dtype=torch.int16, device=DEV)
    tq_native.act_encode(x, True, 0.02, 9, 3, codes)
    ho = (hw + pt + (1 if s == 2 and pt == 0 else 1) - 3) // s + 1
    sc = torch.rand(c, dtype=torch.float64, device=DEV) * 1e-5
    sh = torch.randn(c, dtype=torch.float64, device=DEV) * 0.1
    outs = []
    # (sliding-window mode, streaming mode, blocks per streaming segment)
    for mode, stream, seg in (("0", "0", "0"), ("4", "0", "0"), ("8", "0", "0"),
                              ("4", "1", "0"), ("4", "1", "3"), ("4", "8", "2"), ("4", "2", "3")):
        monkeypatch.setenv("TQ_DW_SLIDE", mode)
        monkeypatch.setenv("TQ_DW_STREAM", stream)
        monkeypatch.setenv("TQ_DW_SEG", seg)
        o = torch.full((3, c, ho, ho), float("nan"), device=DEV).contiguous(
            memory_format=torch.channels_last)
        nc = torch.full((3, ho, ho, cp), -1, dtype=torch.int16, device=DEV)
        tq_native.dwconv2d_termpair_fused(codes, c, layer.w_codes, 3, 3, (s, s), (pt, pl),
                                          (1, 1), ho, ho, sc, sh, relu, out=o, next_codes=nc,
                                          quant=(0.03, 9, 3))
        outs.append((o.view(torch.int32).cpu(), nc.cpu()))
    for o, nc in outs[1:]:
        assert torch.equal(o, outs[0][0]) and torch.equal(nc, outs[0][1])
    assert not torch.isnan(outs[0][0].view(torch.float32)).any()


@pytest.mark.parametrize("cfg", [
    # c, hw, stride, (pad top, pad left), ho: 5x5 pad 2 (EfficientNet stride 1), static-same
    # stride 2 on even / odd inputs (pad 1 before, 2 / 1 after), partial channel chunks
    (40, 28, 1, (2, 2), 28), (120, 14, 1, (2, 2), 14), (240, 28, 2, (1, 1), 14),
    (144, 15, 2, (2, 2), 8), (20, 9, 1, (2, 2), 9), (672, 7, 1, (2, 2), 7),
])
@pytest.mark.parametrize("relu", [6, "swish"])
def test_dw5_streaming_kernel_bit_identical(cfg, relu, monkeypatch):
    """The streaming depthwise kernel at 5x5 (two channels per lane, one or two output rows per
    block, one- and multi-block segments) against the row-blocked 5x5 kernel (TQ_DW_STREAM=0):
    bit-identical fp32 outputs and next-layer codes, for stride 1 and static-same stride 2."""
    import tq_native
    c, hw, s, (pt, pl), ho = cfg
    torch.manual_seed(c + hw + 5)
    conv = nn.Conv2d(c, c, 5, s, 2, groups=c, bias=False)
    layer = tr_layer.TRConv2dLayer(conv.to(DEV), 9, 3, 16, 1, 16)
    cp = layer.act_channels
    x = torch.relu(torch.randn(3, c, hw, hw, device=DEV)).contiguous(
        memory_format=torch.channels_last)
    codes = torch.zeros((3, hw, hw, cp), dtype=torch.int16, device=DEV)
    tq_native.act_encode(x, True, 0.02, 9, 3, codes)
    sc = torch.rand(c, dtype=torch.float64, device=DEV) * 1e-5
    sh = torch.randn(c, dtype=torch.float64, device=DEV) * 0.1
    outs = []
    monkeypatch.setenv("TQ_DW_STREAM5", "1")
    for stream, seg in (("0", "0"), ("1", "0"), ("1", "3"), ("8", "0"), ("8", "2")):
        monkeypatch.setenv("TQ_DW_STREAM", stream)
        monkeypatch.setenv("TQ_DW_SEG", seg)
        o = torch.full((3, c, ho, ho), float("nan"), device=DEV).contiguous(
            memory_format=torch.channels_last)
        nc = torch.full((3, ho, ho, cp), -1, dtype=torch.int16, device=DEV)
        tq_native.dwconv2d_termpair_fused(codes, c, layer.w_codes, 5, 5, (s, s), (pt, pl),
                                          (1, 1), ho, ho, sc, sh, relu, out=o, next_codes=nc,
                                          quant=(0.03, 9, 3))
        outs.append((o.view(torch.int32).cpu(), nc.cpu()))
    for o, nc in outs[1:]:
        assert torch.equal(o, outs[0][0]) and torch.equal(nc, outs[0][1])
    assert not torch.isnan(outs[0][0].view(torch.float32)).any()


@pytest.mark.parametrize("cfg", [
    # c, k, hw, stride, (pad top, pad left), ho: MobileNet-V2 / EfficientNet-b0 shapes, pad
    # channels (c 20 -> cp 24), static-same stride 2
    (32, 3, 14, 1, (1, 1), 14), (144, 3, 28, 2, (1, 1), 14), (20, 3, 9, 1, (1, 1), 9),
    (40, 5, 28, 1, (2, 2), 28), (240, 5, 28, 2, (1, 1), 14), (20, 5, 9, 1, (2, 2), 9),
])
@pytest.mark.parametrize("form", ["relu6_codes", "relu_codes", "swish_out"])
def test_dw_fast_epilogue_bit_identical(cfg, form, monkeypatch):
    """The streaming depthwise kernel's specialised epilogues (dw_emit_coef FAST: ReLU / ReLU6
    with table codes only, swish with the fp32 output only -- the fused executors' forms)
    against its generic epilogue (TQ_DW_FAST=0): bit-identical codes / outputs."""
    import tq_native
    c, k, hw, s, (pt, pl), ho = cfg
    torch.manual_seed(c + hw + k)
    conv = nn.Conv2d(c, c, k, s, k // 2, groups=c, bias=False)
    layer = tr_layer.TRConv2dLayer(conv.to(DEV), 9, 3, 16, 1, 16)
    cp = layer.act_channels
    x = torch.relu(torch.randn(3, c, hw, hw, device=DEV)).contiguous(
        memory_format=torch.channels_last)
    codes = torch.zeros((3, hw, hw, cp), dtype=torch.int16, device=DEV)
    tq_native.act_encode(x, True, 0.02, 9, 3, codes)
    sc = torch.rand(c, dtype=torch.float64, device=DEV) * 1e-5
    sh = torch.randn(c, dtype=torch.float64, device=DEV) * 0.1
    act = {"relu6_codes": 6, "relu_codes": True, "swish_out": "swish"}[form]
    outs = []
    for fast in ("1", "0"):
        monkeypatch.setenv("TQ_DW_FAST", fast)
        o = nc = None
        if form == "swish_out":
            o = torch.full((3, c, ho, ho), float("nan"), device=DEV).contiguous(
                memory_format=torch.channels_last)
        else:
            nc = torch.full((3, ho, ho, cp), -1, dtype=torch.int16, device=DEV)
        tq_native.dwconv2d_termpair_fused(codes, c, layer.w_codes, k, k, (s, s), (pt, pl),
                                          (1, 1), ho, ho, sc, sh, act, out=o, next_codes=nc,
                                          quant=(0.03, 9, 3))
        outs.append(o.view(torch.int32).cpu() if o is not None else nc.cpu())
    assert torch.equal(outs[0], outs[1])
    if form != "swish_out":
        assert (outs[0] != -1).all()  # every code written, pad channels included


@pytest.mark.parametrize("seed", range(12))
def test_depthwise_termpair_random_sweep(seed):
    """Seeded random depthwise convs (channels 1-200, kernel 3/5, stride 1/2, padding or
    EfficientNet static "same", bias, NCHW / channels_last, odd maps) against the fp64
    depthwise conv of the oracle's TR'd tensors."""
    rng = np.random.default_rng(3000 + seed)
    c = int(rng.integers(1, 201))
    k = int(rng.choice([3, 5]))
    s = int(rng.choice([1, 2]))
    same = bool(rng.random() < 0.3)
    p = int(rng.integers(0, k // 2 + 1))
    hw = int(rng.integers(k, 21))
    bias = bool(rng.random() < 0.5)
    torch.manual_seed(3000 + seed)
    if same:
        conv = Conv2dStaticSamePadding(c, c, k, stride=s, groups=c, bias=bias, image_size=hw)
    else:
        conv = nn.Conv2d(c, c, k, s, p, groups=c, bias=bias)
    w = conv.weight.detach().clone()
    b = conv.bias.detach().clone() if bias else None
    layer = tr_layer.TRConv2dLayer(conv.to(DEV), 9, 3, 16, 1, 16)
    assert layer.mode == "depthwise"
    layer.input_quant.tracking = False
    layer.input_quant.sf = 0.02
    x = torch.relu(torch.randn(int(rng.integers(1, 4)), c, hw, hw))
    xd = x.to(DEV)
    if rng.random() < 0.5:
        xd = xd.to(memory_format=torch.channels_last)
    with torch.no_grad():
        y = layer(xd)
    xq = _tr_x(x, 0.02, 9, 3)
    wq = torch.from_numpy(oracle.tr(w.numpy(), layer.w_sf, 16, 1, 16)).double()
    if same:
        xq = conv.static_padding.cpu()(xq)
    ref = F.conv2d(xq, wq, b.double() if bias else None, s, conv.padding, 1, c)
    mag = F.conv2d(xq.abs(), wq.abs(), None, s, conv.padding, 1, c)
    assert y.shape == ref.shape
    _check(y, ref, mag)


@pytest.mark.parametrize("seed", range(12))
def test_linear_termpair_random_sweep(seed):
    """Seeded random TRLinearLayer(quantize_input=True) shapes (in 1-700, out 1-400, 2-D / 3-D
    inputs) and TR settings (group 1-16, kept terms, data terms) against xq @ wq^T + b in
    fp64 with the oracle's TR'd operands."""
    rng = np.random.default_rng(4000 + seed)
    fin, fout = int(rng.integers(1, 701)), int(rng.integers(1, 401))
    g = int(rng.choice([1, 2, 4, 8, 16]))
    k = int(rng.integers(1, 2 * g + 2))
    dt = int(rng.integers(1, 9))
    torch.manual_seed(4000 + seed)
    lin = nn.Linear(fin, fout)
    w = lin.weight.detach().clone()
    b = lin.bias.detach().clone()
    layer = tr_layer.TRLinearLayer(lin.to(DEV), 8, dt, 8, g, k, quantize_input=True)
    assert layer.termpair
    layer.input_quant.tracking = False
    layer.input_quant.sf = 0.01
    shape = (int(rng.integers(1, 40)), fin) if rng.random() < 0.5 else \
        (int(rng.integers(1, 12)), int(rng.integers(1, 12)), fin)
    x = torch.randn(*shape)
    with torch.no_grad():
        y = layer(x.to(DEV))
    xq = _tr_x(x, 0.01, 8, dt)
    wq = torch.from_numpy(oracle.tr(w.numpy(), layer.w_sf, 8, g, k)).double()
    ref = xq @ wq.t() + b.double()
    mag = xq.abs() @ wq.abs().t()
    assert y.shape == shape[:-1] + (fout,)
    _check(y, ref, mag)
