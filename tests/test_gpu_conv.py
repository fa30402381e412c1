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


def _run(n, c, h, w_, cout, ksz, stride, padding, dilation, bias, channels_last, seed,
         db=9, dt=3, wb=9, g=8, k=12):
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
def test_termpair_conv_matches_reference(cfg, channels_last):
    _run(*cfg, channels_last=channels_last, seed=hash(cfg) % 1000)


def test_termpair_conv_group_sizes():
    for g, k in [(1, 9), (2, 3), (16, 24), (32, 48)]:
        _run(2, 64, 8, 8, 64, 3, 1, 1, 1, False, True, seed=g, g=g, k=k)


def test_act_codes_bit_exact():
    torch.manual_seed(9)
    x = torch.randn(2, 40, 6, 5, device=DEV)
    for fmt in (torch.contiguous_format, torch.channels_last):
        xi = x.to(memory_format=fmt)
        codes = torch.empty((2, 6, 5, 40), dtype=torch.int16, device=DEV)
        import tq_native
        nhwc = fmt == torch.channels_last
        tq_native.act_encode(xi, nhwc, 0.01, 9, 3, codes)
        exp = oracle.tr(x.cpu().numpy().reshape(1, -1, 1, 1), 0.01, 9, 1, 3).reshape(x.shape)
        exp_codes = np.rint(exp / np.float32(0.01)).astype(np.int64)
        assert torch.equal(codes.cpu().long().permute(0, 3, 1, 2),
                           torch.from_numpy(exp_codes))


def test_termpair_resnet_layer1_full_batch():
    """A ResNet-18 layer1 conv at the bench batch (256x64x56x56), checked on 4 images."""
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(64, 64, 3, 1, 1, bias=False)
    torch.nn.init.kaiming_normal_(conv.weight, mode='fan_out', nonlinearity='relu')
    w = conv.weight.detach().clone()
    layer = tr_layer.TRConv2dLayer(conv.to(DEV), 9, 3, 9, 8, 12)
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
