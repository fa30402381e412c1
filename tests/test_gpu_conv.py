"""GPU parity of the term-pair Conv2d against conv2d of the oracle's TR'd tensors.

Reference: y_ref = conv2d_fp64(TR(x), TR(w)) + bias, with TR from the oracle and the TR'd
tensors exactly the reference's fake-quantized fp32 values.  The term-pair kernel must match
within the north star's 1e-5 relative bound (SURVEY 8(d) "Output parity"):
    |y - y_ref| <= 1e-5 * max(|y_ref|, sum_k |x_hat_k| |w_hat_k|)   per element
(the second term guards cancellation).  The integer term sums are checked bit-exactly."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import oracle
import tq_ops
import tr_layer

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
RTOL = 1e-5


def _ref(x, w, bias, sf_x, sf_w, db, dt, wb, g, k, stride, padding, dilation):
    xq = torch.from_numpy(oracle.tr(x.contiguous().view(1, -1, 1, 1).cpu().numpy(), sf_x, db,
                                    1, dt)).view(x.shape)
    wq = torch.from_numpy(oracle.tr(w.cpu().numpy(), sf_w, wb, g, k))
    b64 = bias.double().cpu() if bias is not None else None
    y = F.conv2d(xq.double(), wq.double(), b64, stride, padding, dilation)
    mag = F.conv2d(xq.double().abs(), wq.double().abs(), None, stride, padding, dilation)
    return y, mag, wq


@pytest.fixture(params=["mfma", "valu"])
def engine(request, monkeypatch):
    monkeypatch.setenv("TQ_CONV_ENGINE", request.param)
    return request.param


def _run(n, c, h, w_, cout, ksz, stride, padding, dilation, bias, channels_last, seed,
         db=9, dt=3, wb=9, g=8, k=12, engine=None):
    gen = torch.Generator().manual_seed(seed)
    x = torch.relu(torch.randn(n, c, h, w_, generator=gen))
    w = torch.randn(cout, c, ksz, ksz, generator=gen) * 0.05
    b = torch.randn(cout, generator=gen) if bias else None
    conv = torch.nn.Conv2d(c, cout, ksz, stride, padding, dilation, bias=bias)
    with torch.no_grad():
        conv.weight.copy_(w)
        if bias:
            conv.bias.copy_(b)
    layer = tr_layer.TRConv2dLayer(conv.to(DEV), db, dt, wb, g, k)
    assert layer.termpair
    if engine is not None:
        assert layer.engine == engine
        assert layer.w_codes.dtype == (torch.float16 if engine == "mfma" else torch.int16)
    layer.input_quant.tracking = False
    layer.input_quant.sf = 0.02
    xd = x.to(DEV)
    if channels_last:
        xd = xd.to(memory_format=torch.channels_last)
    with torch.no_grad():
        y = layer(xd)
    assert y.shape == (n, cout, (h + 2 * padding - dilation * (ksz - 1) - 1) // stride + 1,
                       (w_ + 2 * padding - dilation * (ksz - 1) - 1) // stride + 1)
    if channels_last:
        assert y.is_contiguous(memory_format=torch.channels_last)
    y_ref, mag, wq = _ref(x, w, b, 0.02, layer.w_sf, db, dt, wb, g, k, stride, padding,
                          dilation)
    # the layer's weight parameter is the reference's fake-quantized weight, bit for bit
    assert torch.equal(layer.conv.weight.detach().cpu(), wq)
    err = (y.double().cpu() - y_ref).abs()
    bound = RTOL * torch.maximum(y_ref.abs(), mag) + 1e-30
    assert bool((err <= bound).all()), float((err / bound).max())
    return y, y_ref


@pytest.mark.parametrize("cfg", [
    # n, c, h, w, cout, k, stride, pad, dil, bias
    (2, 64, 14, 14, 64, 3, 1, 1, 1, False),
    (2, 64, 15, 15, 128, 3, 2, 1, 1, False),
    (2, 64, 14, 14, 128, 1, 2, 0, 1, False),
    (1, 128, 7, 7, 256, 3, 1, 1, 1, True),
    (3, 24, 9, 11, 40, 3, 1, 1, 1, True),      # C % 8 == 0, Cout % 64 != 0
    (2, 20, 8, 8, 36, 3, 1, 2, 2, False),     # padded channels, dilation 2
    (1, 3, 16, 16, 10, 5, 2, 2, 1, True),     # C = 3
    (2, 256, 7, 7, 512, 3, 2, 1, 1, False),
    (1, 512, 7, 7, 512, 3, 1, 1, 1, False),
])
@pytest.mark.parametrize("channels_last", [False, True])
def test_termpair_conv_matches_reference(cfg, channels_last, engine):
    _run(*cfg, channels_last=channels_last, seed=hash(cfg) % 1000, engine=engine)


def test_termpair_conv_group_sizes(engine):
    for g, k in [(1, 9), (2, 3), (16, 24), (32, 48)]:
        _run(2, 64, 8, 8, 64, 3, 1, 1, 1, False, True, seed=g, g=g, k=k, engine=engine)


@pytest.mark.parametrize("dtype", [torch.int16, torch.float16])
def test_act_codes_bit_exact(dtype):
    import tq_native
    torch.manual_seed(9)
    x = torch.randn(2, 40, 6, 5, device=DEV)
    for fmt in (torch.contiguous_format, torch.channels_last):
        xi = x.to(memory_format=fmt)
        codes = torch.empty((2, 6, 5, 40), dtype=dtype, device=DEV)
        nhwc = fmt == torch.channels_last
        tq_native.act_encode(xi, nhwc, 0.01, 9, 3, codes)
        exp = oracle.tr(x.cpu().numpy().reshape(1, -1, 1, 1), 0.01, 9, 1, 3).reshape(x.shape)
        exp_codes = np.rint(exp / np.float32(0.01)).astype(np.int64)
        got = codes.cpu().double()
        assert torch.equal(got, got.round())  # fp16 codes are exact integers
        assert torch.equal(got.long().permute(0, 3, 1, 2), torch.from_numpy(exp_codes))


def _engines_pair(cin, cout, ksz, stride, pad, x, db, dt, wb, g, k, sf_x, w=None, seed=0,
                  dil=1):
    """The same layer built on both engines, run on x; returns (mfma layer, y_mfma, y_valu)."""
    import os
    torch.manual_seed(seed)
    conv = torch.nn.Conv2d(cin, cout, ksz, stride, pad, dil, bias=True)
    if w is not None:
        with torch.no_grad():
            conv.weight.copy_(w)
    outs, layers = [], []
    old = os.environ.get("TQ_CONV_ENGINE")
    try:
        for eng in ("mfma", "valu"):
            os.environ["TQ_CONV_ENGINE"] = eng
            lay = tr_layer.TRConv2dLayer(copy_conv(conv).to(DEV), db, dt, wb, g, k)
            assert lay.engine == eng
            lay.input_quant.tracking = False
            lay.input_quant.sf = sf_x
            with torch.no_grad():
                outs.append(lay(x).cpu())
            layers.append(lay)
    finally:
        if old is None:
            os.environ.pop("TQ_CONV_ENGINE", None)
        else:
            os.environ["TQ_CONV_ENGINE"] = old
    return layers[0], outs[0], outs[1]


def copy_conv(conv):
    import copy
    return copy.deepcopy(conv)


@pytest.mark.parametrize("layer", [1, 5, 7, 10, 16])
def test_mfma_engine_bit_identical_to_valu(layer):
    """Both engines sum the same integers exactly, so outputs match bit for bit (ResNet-18
    TR layer shapes, odd batch: partial tiles)."""
    from conftest import RESNET18_TR
    cin, cout, ksz, s, hin = RESNET18_TR[layer - 1]
    torch.manual_seed(layer)
    x = torch.relu(torch.randn(3, cin, hin, hin, device=DEV)).to(
        memory_format=torch.channels_last)
    lay, ym, yv = _engines_pair(cin, cout, ksz, s, ksz // 2, x, 9, 3, 9, 8, 12, 0.02,
                                seed=layer)
    assert lay.kc_steps >= 0
    assert torch.equal(ym, yv)


@pytest.mark.parametrize("shape", [
    # n, cin, h, w, cout, k, pad, dil -- stride 1: the MFMA input-patch engine
    (37, 128, 5, 5, 96, 3, 1, 1),    # tiles span many images, 2 channel chunks, Cout % 128
    (3, 64, 9, 11, 64, 5, 2, 1),     # 5x5 taps, one chunk (single patch buffer)
    (2, 192, 13, 7, 128, 3, 2, 2),   # dilation 2, 3 chunks, non-square
    (4, 64, 6, 6, 32, 3, 0, 1),      # no padding, Cout < 64
    (5, 256, 14, 14, 256, 3, 1, 1),  # ResNet layer3 shape
    (9, 512, 7, 7, 512, 3, 1, 1),    # ResNet layer4 shape
])
def test_mfma_patch_engine_bit_identical_to_valu(shape):
    n, cin, h, w_, cout, ksz, pad, dil = shape
    torch.manual_seed(sum(shape))
    x = torch.relu(torch.randn(n, cin, h, w_, device=DEV)).to(memory_format=torch.channels_last)
    lay, ym, yv = _engines_pair(cin, cout, ksz, 1, pad, x, 9, 3, 9, 8, 12, 0.02,
                                seed=sum(shape), dil=dil)
    assert torch.equal(ym, yv)


@pytest.mark.parametrize("shape", [
    # n, cin, h, w, cout, stride -- 1x1 convs with Cp % 64 != 0: the direct engine's
    # zero-padded last K-step (MobileNet-V2 / EfficientNet-b0 expand and project shapes)
    (3, 24, 14, 14, 144, 1),
    (2, 96, 9, 9, 24, 1),
    (2, 144, 8, 8, 40, 2),
    (1, 160, 7, 7, 960, 1),
    (4, 40, 5, 5, 240, 1),
    (2, 8, 6, 6, 16, 1),
])
def test_mfma_direct_1x1_partial_chunk_bit_identical_to_valu(shape):
    n, cin, h, w_, cout, s = shape
    torch.manual_seed(sum(shape))
    x = torch.relu(torch.randn(n, cin, h, w_, device=DEV)).to(memory_format=torch.channels_last)
    lay, ym, yv = _engines_pair(cin, cout, 1, s, 0, x, 9, 3, 9, 8, 12, 0.02, seed=sum(shape))
    assert lay.w_codes.shape[1] % 64 == 0
    assert torch.equal(ym, yv)


def test_mfma_flush_window_exact_at_extremes():
    """Saturated activations (every code 511) against constant maximal weights (every code
    256): one K-step of products is 2^23, so the fp32 accumulators must be flushed every 2
    K-steps; the 4608-deep sums (6.0e8) must still match the VALU engine bit for bit."""
    cin, cout = 512, 128
    w = torch.full((cout, cin, 3, 3), 0.01)
    w[::2] *= -1.0
    x = torch.full((2, cin, 7, 7), 100.0, device=DEV).to(memory_format=torch.channels_last)
    lay, ym, yv = _engines_pair(cin, cout, 3, 1, 1, x, 9, 3, 9, 1, 9, 0.02, w=w)
    assert lay.kc_steps == 2
    assert torch.equal(ym, yv)
    assert ym.abs().max().item() > 2**24 * 0.02 * lay.w_sf


def test_termpair_resnet_layer1_full_batch(engine):
    """A ResNet-18 layer1 conv at the bench batch (256x64x56x56), checked on 4 images."""
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(64, 64, 3, 1, 1, bias=False)
    torch.nn.init.kaiming_normal_(conv.weight, mode='fan_out', nonlinearity='relu')
    w = conv.weight.detach().clone()
    layer = tr_layer.TRConv2dLayer(conv.to(DEV), 9, 3, 9, 8, 12)
    assert layer.engine == engine
    layer.input_quant.tracking = False
    layer.input_quant.sf = 0.01
    x = torch.relu(torch.randn(256, 64, 56, 56, device=DEV)).to(
        memory_format=torch.channels_last)
    with torch.no_grad():
        y = layer(x)
    idx = [0, 77, 191, 255]
    y_ref, mag, _ = _ref(x[idx].cpu(), w, None, 0.01, layer.w_sf, 9, 3, 9, 8, 12, 1, 1, 1)
    err = (y[idx].double().cpu() - y_ref).abs()
    assert bool((err <= RTOL * torch.maximum(y_ref.abs(), mag) + 1e-30).all())


@pytest.mark.parametrize("seed", range(16))
def test_termpair_conv_random_sweep(seed, engine):
    """Seeded random conv shapes (kernel 1-7, stride 1-2, padding, dilation 1-2, ragged
    channels, bias, NCHW / channels_last) and TR settings (group 1-32, kept terms, data
    terms) through both engines, each within the 1e-5 bound of conv2d of the oracle's TR'd
    tensors."""
    rng = np.random.default_rng(2000 + seed)
    ksz = int(rng.choice([1, 3, 5, 7]))
    dil = int(rng.choice([1, 1, 2])) if ksz > 1 else 1
    stride = int(rng.choice([1, 2]))
    pad = int(rng.integers(0, ksz // 2 * dil + 1))
    span = dil * (ksz - 1) + 1
    h = int(rng.integers(max(span - 2 * pad, 1), 16))
    w_ = int(rng.integers(max(span - 2 * pad, 1), 16))
    c = int(rng.integers(1, 97))
    cout = int(rng.integers(1, 97))
    g = int(rng.choice([1, 2, 4, 8, 16, 32]))
    k = int(rng.integers(1, 2 * g + 2))
    dt = int(rng.integers(1, 5))
    _run(int(rng.integers(1, 4)), c, h, w_, cout, ksz, stride, pad, dil, bool(rng.random() < 0.5),
         bool(rng.random() < 0.5), seed=seed, dt=dt, g=g, k=k, engine=engine)
