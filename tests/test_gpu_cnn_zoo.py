"""The reference's other CNNs on the term-pair engines: vgg16_bn and alexnet
(reference cnn_models/__init__.py:18-19), converted with static_conv_layer_settings at
(wb=9, g=8, k=12, db=9, dt=3) and calibrated as evaluate_cnn.py does (one tracking pass).

Every converted conv (all but the first, which the reference keeps fp32:
cnn_models/__init__.py:34-36) runs its MFMA term-pair kernel on a 2-image 224x224 batch, and
each output
must be within 1e-5 of the fp64 conv2d(TR(x), TR(w)) + bias of the layer's own input (TR by the
oracle), relative to max(|y|, conv2d(|TR(x)|, |TR(w)|)): the bound every other term-pair test
uses.  VGG16-bn's term-pair MAC count must equal the published results/vgg16_bn-results.json
value for k = 12 (reference profile_model.py:8-46)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import cnn_models
import oracle
import profile_model
import tr_layer
from test_host import PUBLISHED

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _fp64_conv(x, w, b, conv):
    """fp64 conv2d on the GPU (torch's native im2col path; MIOpen has no fp64 convs)."""
    with torch.backends.cudnn.flags(enabled=False):
        return F.conv2d(x.to(DEV), w.to(DEV), None if b is None else b.to(DEV), conv.stride,
                        conv.padding, conv.dilation).cpu()


@pytest.mark.parametrize("arch", ["vgg16_bn", "alexnet"])
def test_zoo_convs_on_term_pair_engines(arch):
    torch.manual_seed(0)
    model = getattr(cnn_models, arch)(pretrained=False).to(DEV).eval()
    settings = cnn_models.static_conv_layer_settings(model, 9, 8, 12)
    q = cnn_models.convert_model(model, settings, 9, 3)
    layers = [m for m in q.modules() if isinstance(m, tr_layer.TRConv2dLayer)]
    assert len(layers) == len(settings) - 1  # the first conv stays an nn.Conv2d
    x = torch.randn(2, 3, 224, 224, device=DEV)
    with torch.no_grad():
        q(x)  # calibration (tracking) pass, as evaluate_cnn.py's first batches
    tr_layer.set_tr_tracking(q, False)
    if arch == "vgg16_bn":
        tmacs, _ = profile_model.get_model_ops(q, (x[:1],))
        assert tmacs == PUBLISHED["vgg16_bn-results.json"]["tr-data3"]["tmacs"][2]
    seen = []

    def hook(mod, inp, out):
        seen.append((mod, inp[0].detach().float().cpu(), out.detach().float().cpu()))
    hs = [m.register_forward_hook(hook) for m in layers]
    with torch.no_grad():
        q(x)
    for h in hs:
        h.remove()
    assert len(seen) == len(layers)
    modes = set()
    for mod, xin, y in seen:
        modes.add(mod.mode)
        assert mod.mode == "termpair", mod.mode
        c = mod.conv
        qd = mod.input_quant
        xq = torch.from_numpy(oracle.tr(xin.numpy().reshape(1, -1, 1, 1), qd.sf, qd.data_bits,
                                        1, qd.data_terms)).view(xin.shape).double()
        w = c.weight.detach().double().cpu()  # the TR'd weight (what the kernels multiply)
        b = c.bias.detach().double().cpu() if c.bias is not None else None
        ref = _fp64_conv(xq, w, b, c)
        mag = _fp64_conv(xq.abs(), w.abs(), None, c)
        bound = 1e-5 * torch.maximum(ref.abs(), mag) + 1e-30
        err = (y.double() - ref).abs()
        assert bool((err <= bound).all()), (arch, tuple(c.weight.shape),
                                            float((err / bound).max()))
    assert modes == {"termpair"}
