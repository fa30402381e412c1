"""GPU parity of the fused MobileNet-V2 executor (tq_fuse.FusedMobileNetV2), teacher forced
layer by layer as tests/test_gpu_fused_parity.py does for ResNet-18: for every term-pair and
depthwise layer of a converted, calibrated MobileNet-V2 (cnn_models/__init__.py:31-58:
depthwise at (16, 1, 16), the rest g=8 k=12 wb=db=9 dt=3), on a sample of images,
  (i)  its input codes are bit-exact oracle.tr() of the fp32 tensor they encode (the
       producer's stored output; channel padding zero), and
  (ii) its fp32 output is within 1e-5 of the fp64 composition conv -> BN -> (ReLU6 |
       + identity) of those same codes (tr_layer.py:124-126 + torchvision's block).
The bench-mode logits are bit-identical to the capture-mode ones."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import cnn_models
import oracle
import tq_fuse
import tr_layer

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SAMPLE = [0, 5]


def _nchw(t, idx):
    return t[idx].double().cpu().contiguous()


def _codes(t, idx, c):
    return t[idx][..., :c].double().permute(0, 3, 1, 2).cpu().contiguous()


def _bn(bn, z):
    a = bn.weight.detach().double().cpu() / torch.sqrt(bn.running_var.double().cpu() + bn.eps)
    return ((z - bn.running_mean.double().cpu().view(1, -1, 1, 1)) * a.view(1, -1, 1, 1) +
            bn.bias.detach().double().cpu().view(1, -1, 1, 1)), a


@pytest.fixture(scope="module")
def net():
    torch.manual_seed(0)
    model = cnn_models.mobilenet_v2(pretrained=False).to(DEV).eval()
    with torch.no_grad():  # non-trivial BN statistics (torchvision init leaves them 0 / 1)
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 2.0)
    st = cnn_models.static_conv_layer_settings(model, 9, 8, 12)
    q = cnn_models.convert_model(model, st, 9, 3).to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 224, 224, device=DEV).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        q(x)
    tr_layer.set_tr_tracking(q, False)
    return q, x


def _check_stem(q, x, rec, module_stem):
    """The stem's fused BN + activation + encode pass (tq_act_encode_act): its fp32 output
    within 1e-5 of the module stem (torch BN + activation), its codes bit-exact TR of it."""
    assert rec["kind"] == "stem"
    with torch.no_grad():
        ref = module_stem().double().cpu()
    y = rec["out"].double().cpu()
    scale = ref.abs().amax(dim=(0, 2, 3), keepdim=True) + 1e-30
    assert bool(((y - ref).abs() <= 1e-5 * scale).all())
    sf, db, dt = rec["quant"]
    c = y.shape[1]
    yq = oracle.tr(y.float().numpy().reshape(1, -1, 1, 1), sf, db, 1, dt)
    exp = torch.from_numpy(np.rint(yq.reshape(y.shape) / np.float32(sf)).astype(np.int64))
    got = rec["codes_out"][..., :c].long().cpu().permute(0, 3, 1, 2)
    assert torch.equal(got, exp)


def test_fused_mobilenet_v2_teacher_forced(net):
    q, x = net
    _teacher_forced(q, x, SAMPLE)


def _bench_batch(seed=1):
    torch.manual_seed(seed)
    return torch.randn(256, 3, 224, 224, device=DEV).contiguous(memory_format=torch.channels_last)


def test_fused_mobilenet_v2_teacher_forced_at_bench_size(net):
    """The same layer-by-layer check on the batch the bench times (256 images: the expand
    engine's persistent grid, the depthwise kernel's segment walks and the large-N index math
    of every kernel at the timed size), on images at both ends of both 128-image chunks."""
    q, _ = net
    _teacher_forced(q, _bench_batch(), [0, 127, 128, 255])


def test_fused_mobilenet_v2_bench_size_variants_bit_identical(net, monkeypatch):
    """At 256 images: the bench's two 128-image chunk streams, and the default dispatch against
    the expand engine off (TQ_XP=0) and the generic epilogues (TQ_EPI_FAST=0, TQ_DW_FAST=0) --
    the same logits bit for bit (so the chunked launches the bench times inherit the 256-image
    teacher-forced parity above)."""
    q, _ = net
    x = _bench_batch()
    fused = tq_fuse.FusedMobileNetV2(q)
    with torch.no_grad():
        ref = fused(x).view(torch.int32)
        streams = [torch.cuda.Stream() for _ in range(2)]
        assert torch.equal(fused.forward_streams(x, streams).view(torch.int32), ref)
        for env in ({"TQ_XP": "0"}, {"TQ_EPI_FAST": "0", "TQ_DW_FAST": "0"}):
            for k, v in env.items():
                monkeypatch.setenv(k, v)
            assert torch.equal(fused(x).view(torch.int32), ref), env
            for k in env:
                monkeypatch.delenv(k)
    torch.cuda.synchronize()


def _teacher_forced(q, x, sample):
    fused = tq_fuse.FusedMobileNetV2(q)
    cap = []
    logits_cap = fused(x, capture=cap)
    logits = fused(x)
    assert torch.equal(logits, logits_cap)
    assert len(cap) == 1 + 2 * 17 + 16 + 1  # stem, 17 dw + 17 project + 16 expand, last
    _check_stem(q, x, cap[0], lambda: q.features[0](x))
    for rec in cap[1:]:
        conv = rec["conv"]
        layer = conv.layer
        sf, db, dt = conv.consumer.quant if rec["kind"] == "dw" else conv.quant
        c_in = layer.conv.in_channels
        codes = _codes(rec["codes_in"], sample, c_in)
        # (i) input codes are exact TR codes: v * sf reproduces TR of some fp32 value and every
        # code is a kept-term value of its own quantized magnitude (checked through the
        # producer below: codes_out == TR(out))
        assert bool((rec["codes_in"][sample][..., c_in:] == 0).all()), rec["name"]
        xq = codes * float(np.float32(sf))
        wq = layer.conv.weight.detach().double().cpu()
        c = layer.conv
        groups = c.groups
        z = F.conv2d(xq, wq, None, c.stride, c.padding, c.dilation, groups)
        mag = F.conv2d(xq.abs(), wq.abs(), None, c.stride, c.padding, c.dilation, groups)
        ref, a = _bn(conv.bn, z)
        bound_mag = mag * a.abs().view(1, -1, 1, 1)
        if rec["residual"] is not None:
            r = _nchw(rec["residual"], sample)
            ref = ref + r
            bound_mag = bound_mag + r.abs()
        if rec["relu"] == 6:
            ref = ref.clamp(0, 6)
        y = _nchw(rec["out"], sample)
        err = (y - ref).abs()
        bound = 1e-5 * torch.maximum(ref.abs(), bound_mag) + 1e-30
        assert bool((err <= bound).all()), (rec["name"], float((err / bound).max()))
        # (ii) the codes this layer emitted are bit-exact TR of its stored fp32 output
        if rec["codes_out"] is not None:
            nxt_quant = None
            for cand in cap:
                if cand.get("codes_in") is rec["codes_out"]:
                    cc = cand["conv"]
                    nxt_quant = cc.consumer.quant if cand["kind"] == "dw" else cc.quant
            assert nxt_quant is not None, rec["name"]
            sf2, db2, dt2 = nxt_quant
            co = y.shape[1]
            yq = oracle.tr(y.float().numpy().reshape(1, -1, 1, 1), sf2, db2, 1, dt2)
            exp = np.rint(yq.reshape(y.shape) / np.float32(sf2)).astype(np.int64)
            got = _codes(rec["codes_out"], sample, co).long()
            assert torch.equal(got, torch.from_numpy(exp)), rec["name"]


@pytest.mark.parametrize("nstreams", [2, 4])
def test_fused_mobilenet_v2_stream_split_bit_identical(net, nstreams):
    """forward_streams: the blocks of image chunks on concurrent HIP streams, the stem and
    classifier on the whole batch -- logits bit-identical to forward()."""
    q, x = net
    fused = tq_fuse.FusedMobileNetV2(q)
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    with torch.no_grad():
        ref = fused(x)
        got = fused.forward_streams(x, streams)
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32))


def test_fused_mobilenet_v2_specialised_epilogues_bit_identical(net, monkeypatch):
    """The engines' specialised epilogues (projection convs: the linear form with one
    table-served code output, tq_epilogue.h emit4_linear_lut; ReLU6 / ReLU forms elsewhere)
    give the generic epilogue's logits bit for bit (TQ_EPI_FAST=0)."""
    q, x = net
    fused = tq_fuse.FusedMobileNetV2(q)
    with torch.no_grad():
        fast = fused(x)
        monkeypatch.setenv("TQ_EPI_FAST", "0")
        generic = fused(x)
    torch.cuda.synchronize()
    assert torch.equal(fast.view(torch.int32), generic.view(torch.int32))
