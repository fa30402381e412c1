"""BASELINE configs[4] -- the ResNet-18 (g, alpha) grid of evaluate_group_size.py -- on the
GPU, setting by setting (/root/reference/evaluate_group_size.py:71-88: wb=db=9, dt=3,
g in {1, 2, 8, 16, 32}, k = round(avg * g) for avg in {1, 1.25, 1.5, 2, 3}, so k up to 96).

For every one of the 25 settings, on a 2-image synthetic 224x224 batch:
  (i)   every TR'd conv weight is bit-exact oracle.tr() at that (g, k) -- group top-k with
        up to 96 kept terms over groups of up to 32 channels;
  (ii)  the term-pair MAC count of the converted model equals the published
        results/resnet18-group-size-results.json point (profile_model, evaluate_cnn.py:28-29);
  (iii) the fused executor bench.py times (tq_fuse.FusedResNet), calibrated as
        evaluate_cnn.eval_model calibrates, is teacher-forced conv by conv: its input codes are
        bit-exact oracle.tr() of the fp32 tensor they encode and its fp32 output is within
        1e-5 of the fp64 conv -> BN -> (+identity) -> ReLU of those codes -- which exercises
        the MFMA exactness windows (general and non-negative) at the widest weight-code sums
        of the grid (g=32, k=96).
"""
import json
import os
from copy import deepcopy

import numpy as np
import pytest
import torch

import cnn_models
import oracle
import profile_model
import tq_fuse
import tr_layer
from test_gpu_fused_parity import _check_input_codes, _out, _reference

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
HERE = os.path.dirname(os.path.abspath(__file__))
PUB = json.load(open(os.path.join(HERE, "golden", "published_results.json")))[
    "resnet18-group-size-results.json"]
AVGS = [1.0, 1.25, 1.5, 2.0, 3.0]
SETTINGS = [(g, i, round(a * g)) for g in (1, 2, 8, 16, 32) for i, a in enumerate(AVGS)]


@pytest.fixture(scope="module")
def fp_model():
    torch.manual_seed(0)
    model = cnn_models.resnet18(pretrained=False).to(DEV).eval()
    import util
    x, _ = util.SyntheticImageNet(2, 2, seed=11, device=DEV).batch(0)
    return model, x.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("g,idx,k", SETTINGS, ids=["g%d-k%d" % (g, k) for g, _, k in SETTINGS])
def test_grid_setting(fp_model, g, idx, k):
    model, x = fp_model
    settings = cnn_models.static_conv_layer_settings(model, 9, g, k)
    q = cnn_models.convert_model(model, settings, 9, 3).to(memory_format=torch.channels_last)
    # (i) weights: TR'd by the HIP op, bit-exact against the oracle's greedy selection
    src = dict(model.named_modules())
    layers = [(n, m) for n, m in q.named_modules() if isinstance(m, tr_layer.TRConv2dLayer)]
    assert len(layers) == 19 and all(m.mode == "termpair" for _, m in layers)
    for name, m in layers:
        w0 = src[name].weight.detach().cpu().numpy()
        assert (m.weight_bits, m.group_size, m.num_terms) == (9, g, k)
        exp = oracle.tr(w0, m.w_sf, 9, g, k)
        assert np.array_equal(m.conv.weight.detach().cpu().numpy(), exp), name
    # (ii) term-pair MACs (profiled on a copy, as evaluate_cnn.eval_model does)
    tmacs, _ = profile_model.get_model_ops(deepcopy(q), (torch.randn(1, 3, 224, 224,
                                                                     device=DEV),))
    assert tmacs == PUB[str(g)]["tmacs"][idx]
    # (iii) calibration pass, then the fused executor teacher-forced conv by conv
    with torch.no_grad():
        q(x)
    tr_layer.set_tr_tracking(q, False)
    fused = tq_fuse.FusedResNet(q)
    with torch.no_grad():
        rec = []
        logits = fused(x, capture=rec)
        assert torch.equal(logits, fused(x))
    convs = [r for r in rec if r["name"] != "stem"]
    assert len(convs) == 19
    sample = [0, 1]
    block_out, conv1_out = rec[0]["out"], None
    for r in convs:
        src_t = conv1_out if r["name"].endswith("conv2") else block_out
        _check_input_codes(r, src_t, sample)
        y_ref, bound = _reference(r["conv"], r["codes_in"], r["residual"], sample,
                                  relu=not r["name"].endswith("downsample"))
        err = (_out(r["out"], sample) - y_ref).abs()
        assert bool((err <= bound).all()), "%s: max err / bound %.3g" % (
            r["name"], float((err / bound).max()))
        if r["name"].endswith("conv1"):
            conv1_out = r["out"]
        elif r["name"].endswith("conv2"):
            block_out = r["out"]
