"""GPU parity of the fused EfficientNet-b0 executor (tq_fuse.FusedEfficientNet), teacher forced
layer by layer as tests/test_gpu_fused_mbv2.py does for MobileNet-V2: for every term-pair and
depthwise layer of a converted, calibrated EfficientNet-b0 (cnn_models/__init__.py:31-58:
depthwise and squeeze-excite convs at (16, 1, 16), the rest g=8 k=12 wb=db=9 dt=3), on a
sample of images,
  (i)  its fp32 output is within 1e-5 (x 1.1, swish's Lipschitz bound) of the fp64
       composition conv (static same padding) -> BN -> (swish | + identity) of the very
       codes it consumed (tr_layer.py:124-126 + efficientnet_pytorch's MBConvBlock), and
  (ii) the codes it emitted are bit-exact oracle.tr() of its stored fp32 output -- for the
       expand convs, of the swish the encode pass stored (itself within 1e-6 of the fp64
       swish of the conv output), for the depthwise layers of fp32(gate * output) with the
       squeeze-excite gate (the project conv's input, MBConvBlock.forward:
       x = sigmoid(x_sq) * x).
The bench-mode logits are bit-identical to the capture-mode ones."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import cnn_models
import oracle
import tq_fuse
import tq_ops
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


def _tr_codes(y, quant):
    sf, db, dt = quant
    yq = oracle.tr(y.float().numpy().reshape(1, -1, 1, 1), sf, db, 1, dt)
    return torch.from_numpy(np.rint(yq.reshape(y.shape) / np.float32(sf)).astype(np.int64))


@pytest.fixture(scope="module")
def net():
    torch.manual_seed(0)
    model = cnn_models.efficientnet_b0(pretrained=False).to(DEV).eval()
    with torch.no_grad():  # non-trivial BN statistics
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


def _consumer_quant(cap, codes):
    for cand in cap:
        if cand.get("codes_in") is codes:
            cc = cand["conv"]
            return cc.consumer.quant if cand["kind"] == "dw" else cc.quant
    return None


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


def test_fused_efficientnet_b0_teacher_forced(net):
    q, x = net
    _teacher_forced(q, x, SAMPLE)


def _bench_batch(seed=1):
    torch.manual_seed(seed)
    return torch.randn(256, 3, 224, 224, device=DEV).contiguous(memory_format=torch.channels_last)


def test_fused_efficientnet_b0_teacher_forced_at_bench_size(net):
    """The same layer-by-layer check on the batch the bench times (256 images: the SE gate
    kernel's 256 workgroups, the gate-and-encode pass's fixed-chunk index path, the expand
    engine's persistent grid, the depthwise segment walks), on images at both ends of both
    128-image chunks."""
    q, _ = net
    _teacher_forced(q, _bench_batch(), [0, 127, 128, 255])


def test_fused_efficientnet_b0_bench_size_variants_bit_identical(net, monkeypatch):
    """At 256 images: the bench's two 128-image chunk streams, and the default dispatch against
    the expand engine off (TQ_XP=0), the module-call squeeze-excite (TQ_SE_FUSED=0), the
    gate-and-encode pass's division form (TQ_AEA_FIXED=0) and the generic epilogues
    (TQ_EPI_FAST=0, TQ_DW_FAST=0) -- the same logits bit for bit."""
    q, _ = net
    x = _bench_batch()
    fused = tq_fuse.FusedEfficientNet(q)
    with torch.no_grad():
        ref = fused(x).view(torch.int32)
        streams = [torch.cuda.Stream() for _ in range(2)]
        assert torch.equal(fused.forward_streams(x, streams).view(torch.int32), ref)
        for env in ({"TQ_XP": "0"}, {"TQ_SE_FUSED": "0"}, {"TQ_AEA_FIXED": "0"},
                    {"TQ_EPI_FAST": "0", "TQ_DW_FAST": "0"}):
            for k, v in env.items():
                monkeypatch.setenv(k, v)
            assert torch.equal(fused(x).view(torch.int32), ref), env
            for k in env:
                monkeypatch.delenv(k)
    torch.cuda.synchronize()


def _teacher_forced(q, x, sample):
    fused = tq_fuse.FusedEfficientNet(q)
    cap = []
    logits_cap = fused(x, capture=cap)
    logits = fused(x)
    torch.cuda.synchronize()
    assert torch.equal(logits, logits_cap)
    assert len(cap) == 1 + 16 + 16 + 15 + 1  # stem, dw + project per block, 15 expand, head
    _check_stem(q, x, cap[0], lambda: q._swish(q._bn0(q._conv_stem(x))))
    for rec in cap[1:]:
        conv = rec["conv"]
        layer = conv.layer
        sf = (conv.consumer.quant if rec["kind"] == "dw" else conv.quant)[0]
        c = layer.conv
        c_in = c.in_channels
        assert bool((rec["codes_in"][sample][..., c_in:] == 0).all()), rec["name"]
        xq = _codes(rec["codes_in"], sample, c_in) * float(np.float32(sf))
        top, bottom, left, right = tq_ops.static_padding(c)
        xq = F.pad(xq, (left, right, top, bottom))
        wq = c.weight.detach().double().cpu()
        z = F.conv2d(xq, wq, None, c.stride, c.padding, c.dilation, c.groups)
        mag = F.conv2d(xq.abs(), wq.abs(), None, c.stride, c.padding, c.dilation, c.groups)
        ref, a = _bn(conv.bn, z)
        bound_mag = mag * a.abs().view(1, -1, 1, 1)
        if rec["residual"] is not None:
            r = _nchw(rec["residual"], sample)
            ref = ref + r
            bound_mag = bound_mag + r.abs()
        bound = 1e-5 * torch.maximum(ref.abs(), bound_mag)
        if rec["act"] == "swish":
            ref = ref * torch.sigmoid(ref)
            bound = 1.1 * bound + 1e-6 * ref.abs()
        y = _nchw(rec["out"], sample)
        err = (y - ref).abs()
        assert bool((err <= bound + 1e-30).all()), (rec["name"], float((err / bound).max()))
        if rec.get("post") is not None:  # the swish pass after an expand conv's BN output
            post = _nchw(rec["post"], sample)
            sw = y * torch.sigmoid(y)
            assert bool(((post - sw).abs() <= 1e-6 * sw.abs() + 1e-7 * y.abs() + 1e-30).all()), \
                rec["name"]
            y = post
        if rec["codes_out"] is None:
            continue
        quant = _consumer_quant(cap, rec["codes_out"])
        assert quant is not None, rec["name"]
        co = y.shape[1]
        val = y
        if rec.get("gate") is not None:  # fp32(gate * y), as the module's sigmoid(x_sq) * x
            g = rec["gate"][sample].cpu().float().view(len(sample), co, 1, 1)
            val = (g * y.float()).double()
        got = _codes(rec["codes_out"], sample, co).long()
        assert torch.equal(got, _tr_codes(val, quant)), rec["name"]


def test_fused_efficientnet_b0_matches_module_path(net):
    """Whole network against the module path (the reference composition): the logits agree
    to the accumulated effect of midpoint code flips (a loose end-to-end sanity check; the
    per-layer parity above is the bar)."""
    q, x = net
    fused = tq_fuse.FusedEfficientNet(q)
    with torch.no_grad():
        a = fused(x)
        b = q(x)
    torch.cuda.synchronize()
    rel = ((a - b).norm() / b.norm()).item()
    assert rel < 5e-2, rel


def test_swish_is_torchs_fp32_swish_bit_for_bit():
    """The fused swish (tq_device.h swish_f32: 1 / (1 + expf(-y)) then y * s, the device
    library's expf and an IEEE division) equals the module path's MemoryEfficientSwish,
    x * torch.sigmoid(x) on the GPU, bit for bit -- so codes the fused executor emits after a
    swish are TR of exactly the value the reference composition computes."""
    import tq_native
    torch.manual_seed(3)
    x = torch.randn(4, 64, 17, 9, device=DEV) * 4
    flat = x.view(-1)
    edge = torch.tensor([0.0, -0.0, 1e-30, -1e-30, 88.0, -88.0, 104.0, -104.0, 1e4, -1e4,
                         float("inf"), float("-inf"), 20.0, -20.0, 0.5, -0.5], device=DEV)
    flat[:edge.numel()] = edge
    x = x.contiguous(memory_format=torch.channels_last)
    out = torch.empty_like(x)
    codes = torch.empty((4, 17, 9, 64), dtype=torch.float16, device=DEV)
    tq_native.act_encode_act(x, 0.01, 9, 3, codes, act="swish", out=out)
    ref = x * torch.sigmoid(x)
    torch.cuda.synchronize()
    same = (out.view(torch.int32) == ref.view(torch.int32)) | (torch.isnan(out) & torch.isnan(ref))
    assert bool(same.all()), int((~same).sum())
    yq = oracle.tr(out.permute(0, 2, 3, 1).contiguous().cpu().numpy().reshape(1, -1, 1, 1),
                   0.01, 9, 1, 3)
    exp = np.rint(yq.reshape(4, 17, 9, 64) / np.float32(0.01)).astype(np.int64)
    assert np.array_equal(codes.long().cpu().numpy(), exp)


def test_fused_se_gate_bit_identical_to_module_path(net, monkeypatch):
    """The fused squeeze-excite kernel (tq_se_gate_f32) against the module calls it replaces
    (TRConv2dLayer "wide" reduce / expand convs, torch swish and sigmoid) on every SE block's
    real depthwise output: the gates must be bit-identical (exact int64 term sums, one fp64
    fold each, torch's fp32 swish / sigmoid compositions)."""
    import torch.nn.functional as F
    q, x = net
    fused = tq_fuse.FusedEfficientNet(q)
    with torch.no_grad():
        cap = []
        fused(x, capture=cap)
        checked = 0
        for i, b in enumerate(fused.blocks):
            if not b.has_se:
                continue
            assert b.se is not None, i  # every b0 SE block takes the fused kernel
            rec = next(r for r in cap if r["name"] == "block%d.dw" % i)
            d, g = rec["out"], rec["gate"]
            blk = b.block
            ref = torch.sigmoid(blk._se_expand(blk._swish(blk._se_reduce(
                F.adaptive_avg_pool2d(d, 1))))).reshape(d.shape[0], d.shape[1])
            assert torch.equal(g.view(torch.int32), ref.contiguous().view(torch.int32)), i
            monkeypatch.setenv("TQ_SE_FUSED", "0")
            assert torch.equal(b.gate(d), g), i
            monkeypatch.delenv("TQ_SE_FUSED")
            checked += 1
    assert checked == 16


@pytest.mark.parametrize("nstreams", [2, 4])
def test_fused_efficientnet_b0_stream_split_bit_identical(net, nstreams):
    """forward_streams: the blocks of image chunks on concurrent HIP streams, the stem and
    classifier on the whole batch -- logits bit-identical to forward()."""
    q, x = net
    fused = tq_fuse.FusedEfficientNet(q)
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    with torch.no_grad():
        ref = fused(x)
        got = fused.forward_streams(x, streams)
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32))


def test_fused_efficientnet_b0_specialised_epilogues_bit_identical(net, monkeypatch):
    """The specialised epilogues (projection convs: tq_epilogue.h emit4_linear_lut; the
    expand engine's and depthwise kernel's forms) give the generic epilogues' logits bit for
    bit (TQ_EPI_FAST=0, TQ_DW_FAST=0)."""
    q, x = net
    fused = tq_fuse.FusedEfficientNet(q)
    with torch.no_grad():
        fast = fused(x)
        monkeypatch.setenv("TQ_EPI_FAST", "0")
        monkeypatch.setenv("TQ_DW_FAST", "0")
        generic = fused(x)
    torch.cuda.synchronize()
    assert torch.equal(fast.view(torch.int32), generic.view(torch.int32))
