"""GPU parity of the fused term-pair epilogue (BN fold, residual, ReLU, next-layer TR codes),
its schedules and the stem tail."""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import oracle
import tq_fuse
import tq_native
import tr_layer
import cnn_models

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _layer(cin, cout, k, s, seed):
    torch.manual_seed(seed)
    conv = nn.Conv2d(cin, cout, k, s, k // 2, bias=False)
    nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
    layer = tr_layer.TRConv2dLayer(conv.to(DEV), 9, 3, 9, 8, 12)
    layer.input_quant.tracking = False
    layer.input_quant.sf = 0.03
    bn = nn.BatchNorm2d(cout).to(DEV).eval()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.5, 2.0)
    return layer, bn


@pytest.fixture(params=["mfma", "valu"])
def engine(request, monkeypatch):
    monkeypatch.setenv("TQ_CONV_ENGINE", request.param)
    return request.param


@pytest.mark.parametrize("cfg", [(64, 64, 3, 1, 14), (64, 128, 3, 2, 15), (64, 128, 1, 2, 14),
                                 (128, 256, 3, 1, 7)])
def test_fused_epilogue_matches_reference_composition(cfg, engine):
    cin, cout, k, s, hw = cfg
    layer, bn = _layer(cin, cout, k, s, seed=cin + k)
    conv = tq_fuse._Conv(layer, bn)
    nxt, _ = _layer(cout, cout, 3, 1, seed=99)
    nxt.input_quant.sf = 0.05
    nxt_conv = tq_fuse._Conv(nxt, None)
    torch.manual_seed(7)
    x = torch.relu(torch.randn(2, cin, hw, hw, device=DEV))
    assert conv.code_dtype == (torch.float16 if engine == "mfma" else torch.int16)
    codes = torch.empty((2, hw, hw, conv.cp_in), dtype=conv.code_dtype, device=DEV)
    tq_native.act_encode(x.contiguous(memory_format=torch.channels_last), True, 0.03, 9, 3,
                         codes)
    ho, wo = conv.out_hw(hw, hw)
    res = torch.randn(2, cout, ho, wo, device=DEV).contiguous(memory_format=torch.channels_last)
    y, ca, _ = conv(codes, out=True, residual=res, relu=True, next_a=nxt_conv)
    # reference composition in fp64 from the oracle's TR'd tensors
    xq = torch.from_numpy(oracle.tr(x.cpu().numpy().reshape(1, -1, 1, 1), 0.03, 9, 1,
                                    3)).view(x.shape).double()
    wq = layer.conv.weight.detach().cpu().double()
    z = F.conv2d(xq, wq, None, s, k // 2)
    mag = F.conv2d(xq.abs(), wq.abs(), None, s, k // 2)
    a = (bn.weight.detach().double() / torch.sqrt(bn.running_var.double() + bn.eps)).cpu()
    bnz = (z - bn.running_mean.double().cpu().view(1, -1, 1, 1)) * a.view(1, -1, 1, 1) + \
        bn.bias.detach().double().cpu().view(1, -1, 1, 1)
    ref = torch.relu(bnz + res.double().cpu())
    bound = 1e-5 * (torch.maximum(ref.abs(), mag * a.abs().view(1, -1, 1, 1)) +
                    res.double().abs().cpu()) + 1e-30
    assert bool(((y.double().cpu() - ref).abs() <= bound).all())
    # the emitted codes are exactly TR of the fp32 output the kernel wrote
    yq = oracle.tr(y.contiguous().cpu().numpy().reshape(1, -1, 1, 1), 0.05, 9, 1, 3)
    exp_codes = np.rint(yq.reshape(y.shape) / np.float32(0.05)).astype(np.int64)
    got = ca.cpu().long()[..., :cout].permute(0, 3, 1, 2)
    assert torch.equal(got, torch.from_numpy(exp_codes))


# The executor-vs-module-path comparison lives in tests/test_gpu_fused_parity.py: teacher
# forced, conv by conv, at the bench config (the former whole-network 2e-2 / 75 %-argmax
# check could not tell an epilogue bug from rounding-midpoint code flips).


@pytest.mark.parametrize("sf", [0.0, float("inf"), 1e-38, 1e30])
def test_fused_epilogue_codes_extreme_scales(sf, engine):
    """Next-layer codes at scales outside the fast path's range or at its edges: sf = 0
    (|y|/0 -> maxv, 0/0 -> 0), sf = inf (-> 0), tiny sf (saturates), huge sf (rounds to 0
    or 1 term).  Expected values follow kernels/tr_cuda_kernel.cu:21-23 directly."""
    layer, bn = _layer(64, 64, 3, 1, seed=5)
    conv = tq_fuse._Conv(layer, bn)
    nxt, _ = _layer(64, 64, 3, 1, seed=99)
    nxt.input_quant.sf = sf
    nxt_conv = tq_fuse._Conv(nxt, None)
    torch.manual_seed(8)
    x = torch.relu(torch.randn(2, 64, 9, 9, device=DEV))
    codes = torch.empty((2, 9, 9, conv.cp_in), dtype=conv.code_dtype, device=DEV)
    tq_native.act_encode(x.contiguous(memory_format=torch.channels_last), True, 0.03, 9, 3,
                         codes)
    y, ca, _ = conv(codes, out=True, relu=True, next_a=nxt_conv)
    yn = y.contiguous().cpu().numpy()
    got = ca.cpu().long()[..., :64].permute(0, 3, 1, 2).numpy()
    if sf == float("inf"):
        exp = np.zeros_like(got)
    elif sf == 0.0 or sf == 1e-38:
        exp = np.where(yn > 0, 511, 0)  # TR of maxv = 511 = 512 - 1: two terms, value 511
    else:
        exp = np.rint(oracle.tr(yn.reshape(1, -1, 1, 1), sf, 9, 1, 3).reshape(yn.shape) /
                      np.float32(sf)).astype(np.int64)
    assert (yn > 0).any()
    np.testing.assert_array_equal(got, exp)


def test_fused_resnet_shared_downsample_codes(monkeypatch):
    """A block's conv1 and downsample read one tensor, so their calibrated quantizers agree
    and the executor encodes it once; the result is bit-identical to encoding it twice."""
    torch.manual_seed(0)
    model = cnn_models.resnet18(pretrained=False).to(DEV).eval()
    settings = cnn_models.static_conv_layer_settings(model, 9, 8, 12)
    q = cnn_models.convert_model(model, settings, 9, 3).to(memory_format=torch.channels_last)
    x = torch.randn(4, 3, 224, 224, device=DEV).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        q(x)
    tr_layer.set_tr_tracking(q, False)
    fused = tq_fuse.FusedResNet(q)
    downs = [b for b in fused.blocks if b.down is not None]
    assert downs and all(tq_fuse._same_codes(b.conv1, b.down) for b in downs)
    with torch.no_grad():
        shared = fused(x)
        monkeypatch.setattr(tq_fuse, "_same_codes", lambda a, b: False)
        separate = fused(x)
    assert torch.equal(shared, separate)


@pytest.mark.parametrize("layer,cfgs", [(1, [(2, 1), (2, -1), (6, -1)]),
                                         (6, [(1, 1), (1, -1), (5, -1), (4, -1)]),
                                         (16, [(1, 1), (1, -1), (4, -1), (4, 3)]),
                                         (17, [(1, 1), (1, -1), (3, -1)])])
def test_schedules_are_bit_identical(layer, cfgs, monkeypatch):
    """Data-parallel, K-split (atomics) and stream-K (slab fixup) schedules of the VALU
    engine and both tile configs of the MFMA engine sum the same integers, so every output
    and code must be bit-identical."""
    import tq_ops
    monkeypatch.setenv("TQ_CONV_ENGINE", "valu")
    from conftest import RESNET18_TR
    cin, cout, k, s, hin = RESNET18_TR[layer - 1]
    batch = 37  # odd pixel count: partial last tile
    torch.manual_seed(layer)
    conv = nn.Conv2d(cin, cout, k, s, k // 2, bias=False).to(DEV)
    lay = tr_layer.TRConv2dLayer(conv, 9, 3, 9, 8, 12)
    cp = tq_ops.act_channels(cin)
    x = torch.relu(torch.randn(batch, cin, hin, hin, device=DEV)).to(
        memory_format=torch.channels_last)
    codes = torch.empty((batch, hin, hin, cp), dtype=torch.int16, device=DEV)
    tq_native.act_encode(x, True, 0.02, 9, 3, codes)
    ho = (hin + 2 * (k // 2) - k) // s + 1
    ws = tq_native.conv2d_workspace(batch * ho * ho, cout, DEV)
    sc = torch.rand(cout, dtype=torch.float64, device=DEV) * 1e-4
    sh = torch.randn(cout, dtype=torch.float64, device=DEV)
    outs = []
    for cfg, sp in cfgs:
        o = torch.full((batch, cout, ho, ho), float("nan"), device=DEV).contiguous(
            memory_format=torch.channels_last)
        ca = torch.zeros((batch, ho, ho, tq_ops.act_channels(cout)), dtype=torch.int16,
                         device=DEV)
        tq_native.conv2d_termpair_fused(codes, lay.w_codes, cout, k, k, (s, s),
                                        (k // 2, k // 2), (1, 1), ho, ho, out=o, ch_scale=sc,
                                        ch_shift=sh, relu=True, codes_a=ca,
                                        quant_a=(0.05, 9, 3), workspace=ws, split_k=sp,
                                        config=cfg)
        outs.append((o.cpu(), ca.cpu()))
    monkeypatch.setenv("TQ_CONV_ENGINE", "mfma")
    lay_m = tr_layer.TRConv2dLayer(conv, 9, 3, 9, 8, 12)
    assert lay_m.engine == "mfma" and torch.equal(lay_m.w_codes[:cout, :k * k * cp].float(),
                                                   lay.w_codes[:cout, :k * k * cp].float())
    codes_m = torch.empty((batch, hin, hin, cp), dtype=torch.float16, device=DEV)
    tq_native.act_encode(x, True, 0.02, 9, 3, codes_m)
    for cfg in range(1, tq_native.lib().tq_conv2d_mfma_num_configs() + 1):
        o = torch.full((batch, cout, ho, ho), float("nan"), device=DEV).contiguous(
            memory_format=torch.channels_last)
        ca = torch.zeros((batch, ho, ho, tq_ops.act_channels(cout)), dtype=torch.float16,
                         device=DEV)
        tq_native.conv2d_termpair_fused(codes_m, lay_m.w_codes, cout, k, k, (s, s),
                                        (k // 2, k // 2), (1, 1), ho, ho, out=o, ch_scale=sc,
                                        ch_shift=sh, relu=True, codes_a=ca,
                                        quant_a=(0.05, 9, 3), config=cfg,
                                        kc_steps=lay_m.kc_steps)
        outs.append((o.cpu(), ca.cpu().to(torch.int16)))
    # the wider exactness windows for non-negative (post-ReLU) codes, as the fused executor
    # runs them: still the exact integer sums
    for cfg in range(0, tq_native.lib().tq_conv2d_mfma_num_configs() + 1):
        o = torch.full((batch, cout, ho, ho), float("nan"), device=DEV).contiguous(
            memory_format=torch.channels_last)
        ca = torch.zeros((batch, ho, ho, tq_ops.act_channels(cout)), dtype=torch.float16,
                         device=DEV)
        tq_native.conv2d_termpair_fused(codes_m, lay_m.w_codes, cout, k, k, (s, s),
                                        (k // 2, k // 2), (1, 1), ho, ho, out=o, ch_scale=sc,
                                        ch_shift=sh, relu=True, codes_a=ca,
                                        quant_a=(0.05, 9, 3), config=cfg,
                                        kc_steps=lay_m.kc_steps_nonneg,
                                        kc_chunk=lay_m.kc_chunk_nonneg)
        outs.append((o.cpu(), ca.cpu().to(torch.int16)))
    o0, c0 = outs[0]
    assert not torch.isnan(o0).any()
    for o, c in outs[1:]:
        assert torch.equal(o, o0) and torch.equal(c, c0)


@pytest.mark.parametrize("layer", [1, 7, 11])
def test_signed_code_tables_bit_identical(layer, monkeypatch):
    """The epilogue code tables for values WITHOUT a ReLU (MobileNet-V2 / EfficientNet project
    convs, tq_device.h lut_codes: the table's code of q(|y|), negated for y < 0, NaN -> 0)
    against the VALU engine's computed codes (no tables) and against every MFMA config with the
    tables off (TQ_LUT=0): outputs and codes bit-identical, with negative, zero, NaN and
    infinite values (a residual carries the non-finite ones)."""
    import tq_ops
    from conftest import RESNET18_TR
    cin, cout, k, s, hin = RESNET18_TR[layer - 1]
    batch = 7
    torch.manual_seed(100 + layer)
    conv = nn.Conv2d(cin, cout, k, s, k // 2, bias=False).to(DEV)
    x = torch.relu(torch.randn(batch, cin, hin, hin, device=DEV)).to(
        memory_format=torch.channels_last)
    ho = (hin + 2 * (k // 2) - k) // s + 1
    sc = (torch.rand(cout, dtype=torch.float64, device=DEV) - 0.5) * 2e-4
    sh = torch.randn(cout, dtype=torch.float64, device=DEV) * 0.1
    res = torch.randn(batch, cout, ho, ho, device=DEV).contiguous(
        memory_format=torch.channels_last)
    flat = res.permute(0, 2, 3, 1).view(-1)  # the NHWC storage
    flat[::97] = float("nan")
    flat[1::101] = float("inf")
    flat[2::103] = -float("inf")
    flat[3::107] = 0.0
    flat[4::109] = -0.0

    def run(engine, lut, cfg, fmt):
        monkeypatch.setenv("TQ_CONV_ENGINE", engine)
        monkeypatch.setenv("TQ_LUT", lut)
        lay = tr_layer.TRConv2dLayer(conv, 9, 3, 9, 8, 12)
        cp = tq_ops.act_channels(cin)
        codes = torch.empty((batch, hin, hin, cp), dtype=fmt, device=DEV)
        tq_native.act_encode(x, True, 0.02, 9, 3, codes)
        o = torch.full((batch, cout, ho, ho), 7.0, device=DEV).contiguous(
            memory_format=torch.channels_last)
        ca = torch.zeros((batch, ho, ho, tq_ops.act_channels(cout)), dtype=fmt, device=DEV)
        kw = {} if engine == "valu" else {"kc_steps": lay.kc_steps}
        tq_native.conv2d_termpair_fused(codes, lay.w_codes, cout, k, k, (s, s),
                                        (k // 2, k // 2), (1, 1), ho, ho, out=o, ch_scale=sc,
                                        ch_shift=sh, residual=res, relu=False, codes_a=ca,
                                        quant_a=(0.05, 9, 3), config=cfg, **kw)
        # codes as the signed integer term sums (fp16 codes are exact integers)
        return o.view(torch.int32).cpu(), ca.float().cpu()

    o0, c0 = run("valu", "1", 0, torch.int16)
    assert (c0 < 0).any() and (c0 > 0).any()
    for cfg in range(0, tq_native.lib().tq_conv2d_mfma_num_configs() + 1):
        for lut in ("1", "0"):
            o, c = run("mfma", lut, cfg, torch.float16)
            assert torch.equal(o, o0) and torch.equal(c, c0), (cfg, lut)
    # the emitted codes are TR of the stored fp32 values (the oracle's restatement)
    y = o0.view(torch.float32).permute(0, 2, 3, 1).contiguous()
    ref = torch.from_numpy(oracle.tr(y.numpy(), 0.05, 9, 1, 3)) / 0.05
    assert torch.equal(c0[..., :cout], ref.round())


@pytest.mark.parametrize("layer,batch", [(8, 5), (13, 8), (13, 37), (16, 8), (19, 3)])
@pytest.mark.parametrize("cfg", [0, 7, 8])
def test_patch_streamk_bit_identical(layer, batch, cfg):
    """The input-patch engine's stream-K schedule (split_k=-1: K-step ranges cut across tile
    boundaries, split tiles finished from int32 slabs by their last piece) sums the same
    integers as its data-parallel tiles (split_k=1): outputs and codes bit-identical,
    including ranges that start inside a channel chunk and batches with fewer K-steps than
    workgroups (empty ranges)."""
    import tq_ops
    from conftest import RESNET18_TR
    cin, cout, k, s, hin = RESNET18_TR[layer - 1]
    assert s == 1 and k == 3
    torch.manual_seed(100 + layer)
    conv = nn.Conv2d(cin, cout, k, s, 1, bias=False).to(DEV)
    lay = tr_layer.TRConv2dLayer(conv, 9, 3, 9, 8, 12)
    assert lay.engine == "mfma"
    cp = tq_ops.act_channels(cin)
    x = torch.relu(torch.randn(batch, cin, hin, hin, device=DEV)).to(
        memory_format=torch.channels_last)
    codes = torch.empty((batch, hin, hin, cp), dtype=torch.float16, device=DEV)
    tq_native.act_encode(x, True, 0.02, 9, 3, codes)
    ws = tq_native.conv2d_workspace(batch * hin * hin, cout, DEV)
    sc = torch.rand(cout, dtype=torch.float64, device=DEV) * 1e-4
    sh = torch.randn(cout, dtype=torch.float64, device=DEV)
    res = torch.randn(batch, cout, hin, hin, device=DEV).contiguous(
        memory_format=torch.channels_last)
    outs = []
    for sp in (1, -1, -1):  # twice: the counters must be usable again
        o = torch.full((batch, cout, hin, hin), float("nan"), device=DEV).contiguous(
            memory_format=torch.channels_last)
        ca = torch.zeros((batch, hin, hin, tq_ops.act_channels(cout)), dtype=torch.float16,
                         device=DEV)
        ws.fill_(-7)  # stale slabs/counters must not leak into the sums
        tq_native.conv2d_termpair_fused(codes, lay.w_codes, cout, k, k, (1, 1), (1, 1),
                                        (1, 1), hin, hin, out=o, ch_scale=sc, ch_shift=sh,
                                        residual=res, relu=True, codes_a=ca,
                                        quant_a=(0.05, 9, 3), workspace=ws, split_k=sp,
                                        config=cfg, kc_steps=lay.kc_steps,
                                        kc_chunk=lay.kc_chunk)
        outs.append((o.cpu(), ca.cpu()))
    o0, c0 = outs[0]
    assert not torch.isnan(o0).any()
    for o, c in outs[1:]:
        assert torch.equal(o, o0) and torch.equal(c, c0)


@pytest.mark.parametrize("dtype", [torch.int16, torch.float16])
def test_stem_bn_relu_maxpool_encode(dtype):
    torch.manual_seed(11)
    bn = nn.BatchNorm2d(64).to(DEV).eval()
    with torch.no_grad():
        bn.weight.uniform_(-1.5, 1.5)  # negative scales too: BN before the max
        bn.bias.uniform_(-0.3, 0.3)
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.5, 2.0)
    x = torch.randn(3, 64, 29, 30, device=DEV).contiguous(memory_format=torch.channels_last)
    ref = F.max_pool2d(torch.relu(bn(x)), 3, 2, 1)
    a = bn.weight.double() / torch.sqrt(bn.running_var.double() + bn.eps)
    sc = a.float().contiguous()
    sh = (bn.bias.double() - bn.running_mean.double() * a).float().contiguous()
    out = torch.empty_like(ref, memory_format=torch.channels_last)
    codes = torch.empty((3, ref.shape[2], ref.shape[3], 64), dtype=dtype, device=DEV)
    tq_native.bn_relu_maxpool_encode(x, sc, sh, 3, 2, 1, out, codes_a=codes,
                                     quant_a=(0.05, 9, 3))
    assert torch.allclose(out, ref, rtol=1e-6, atol=1e-6)
    yq = oracle.tr(out.contiguous().cpu().numpy().reshape(1, -1, 1, 1), 0.05, 9, 1, 3)
    exp = np.rint(yq.reshape(out.shape) / np.float32(0.05)).astype(np.int64)
    assert torch.equal(codes.cpu().long().permute(0, 3, 1, 2), torch.from_numpy(exp))


@pytest.mark.parametrize("cin,cout,hw,n", [(64, 128, 28, 3), (128, 256, 14, 2), (256, 512, 7, 5),
                                           (64, 64, 9, 1)])
@pytest.mark.parametrize("kc", [0, 2])
def test_fused_downsample_phase_bit_identical(cin, cout, hw, n, kc, monkeypatch):
    """conv2 with the downsample as a second accumulation phase (tq_conv_epilogue.ds_*) equals
    conv2 with the separate downsample conv's stored identity as its residual, bit for bit:
    fp32 output and next-layer codes (partial pixel tiles, odd batches, a flushing main conv)."""
    monkeypatch.setenv("TQ_CONV_ENGINE", "mfma")
    monkeypatch.setenv("TQ_FUSE_DS", "1")
    conv2_l, bn2 = _layer(cout, cout, 3, 1, seed=cout)
    down_l, bnd = _layer(cin, cout, 1, 2, seed=cin + 1)
    down_l.input_quant.sf = 0.04
    conv2 = tq_fuse._Conv(conv2_l, bn2, nonneg=True)
    if kc:
        conv2.kc_steps = kc  # force the flushing main loop (a smaller window stays exact)
    down = tq_fuse._Conv(down_l, bnd, nonneg=True)
    assert conv2.fusable_downsample(down)
    nxt, _ = _layer(cout, cout, 3, 1, seed=5)
    nxt.input_quant.sf = 0.05
    nxt_conv = tq_fuse._Conv(nxt, None, nonneg=True)
    torch.manual_seed(3)
    mid_x = torch.relu(torch.randn(n, cout, hw, hw, device=DEV))
    in_x = torch.relu(torch.randn(n, cin, 2 * hw, 2 * hw, device=DEV))
    mid = torch.empty((n, hw, hw, conv2.cp_in), dtype=torch.float16, device=DEV)
    tq_native.act_encode(mid_x.contiguous(memory_format=torch.channels_last), True, 0.03, 9, 3,
                         mid)
    dcodes = torch.empty((n, 2 * hw, 2 * hw, down.cp_in), dtype=torch.float16, device=DEV)
    tq_native.act_encode(in_x.contiguous(memory_format=torch.channels_last), True, 0.04, 9, 3,
                         dcodes)
    identity, _, _ = down(dcodes, out=True)
    y_sep, c_sep, _ = conv2(mid, out=True, residual=identity, relu=True, next_a=nxt_conv)
    y_fus, c_fus, _ = conv2(mid, out=True, relu=True, next_a=nxt_conv,
                            downsample=(down, dcodes))
    assert torch.equal(y_sep, y_fus)
    assert torch.equal(c_sep.view(torch.int16), c_fus.view(torch.int16))
    assert (y_fus > 0).any()


def test_fused_resnet_downsample_phase(monkeypatch):
    """The executor with each transition block's downsample fused into its conv2 gives the same
    logits, bit for bit, as with separate downsample launches."""
    monkeypatch.setenv("TQ_CONV_ENGINE", "mfma")
    monkeypatch.setenv("TQ_FUSE_DS", "1")
    torch.manual_seed(0)
    model = cnn_models.resnet18(pretrained=False).to(DEV).eval()
    settings = cnn_models.static_conv_layer_settings(model, 9, 8, 12)
    q = cnn_models.convert_model(model, settings, 9, 3).to(memory_format=torch.channels_last)
    x = torch.randn(6, 3, 224, 224, device=DEV).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        q(x)
    tr_layer.set_tr_tracking(q, False)
    fused = tq_fuse.FusedResNet(q)
    downs = [b for b in fused.blocks if b.down is not None]
    assert len(downs) == 3 and all(b.conv2.fusable_downsample(b.down) for b in downs)
    with torch.no_grad():
        one = fused(x)
        monkeypatch.setenv("TQ_FUSE_DS", "0")
        assert not downs[0].conv2.fusable_downsample(downs[0].down)
        two = fused(x)
    assert torch.equal(one, two)


@pytest.mark.parametrize("act", [None, 6, "swish"])
@pytest.mark.parametrize("gated", [False, True])
@pytest.mark.parametrize("fmt", [torch.int16, torch.float16])
def test_act_encode_act_code_table_bit_identical(act, gated, fmt, monkeypatch):
    """tq_act_encode_act's code table (tq_device.h lut_codes: ReLU6 values and, with swish, a
    gate or no activation, signed ones) against its computed codes (TQ_LUT=0) and against the
    oracle's TR of the activated value: bit-identical codes, with negative, zero, NaN and
    infinite inputs and a channel count that leaves pad channels."""
    n, c, hw = 3, 44, 9
    torch.manual_seed(7)
    x = (torch.randn(n, c, hw, hw, device=DEV) * 3).contiguous(memory_format=torch.channels_last)
    flat = x.permute(0, 2, 3, 1).view(-1)  # the NHWC storage
    flat[::89] = float("nan")
    flat[1::97] = float("inf")
    flat[2::101] = -float("inf")
    flat[3::103] = -0.0
    gate = torch.rand(n, c, device=DEV) if gated else None
    cp = 48
    res = []
    for lut in ("1", "0"):
        monkeypatch.setenv("TQ_LUT", lut)
        codes = torch.full((n, hw, hw, cp), 77, dtype=fmt, device=DEV)
        out = torch.empty_like(x)
        tq_native.act_encode_act(x, 0.05, 9, 3, codes, act=act, gate=gate, out=out)
        res.append((codes.float().cpu(), out.cpu()))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1].view(torch.int32), res[1][1].view(torch.int32))
    v = res[0][1].permute(0, 2, 3, 1).contiguous()
    if gated:
        v = v * gate.cpu()[:, None, None, :]
    ref = torch.from_numpy(oracle.tr(v.numpy(), 0.05, 9, 1, 3)) / 0.05
    assert torch.equal(res[0][0][..., :c], ref.round())
    assert (res[0][0][..., c:] == 0).all()


@pytest.mark.parametrize("c,cp", [(200, 200), (44, 48)])
def test_act_encode_act_fixed_chunk_grid(c, cp, monkeypatch):
    """A grid-stride wide enough that lanes walk several pixels across image boundaries: the
    fixed-chunk loop (grid stride a multiple of the chunks per pixel, image index from a
    reciprocal) gives the per-iteration-division loop's bits (TQ_AEA_FIXED=0)."""
    n, hw = 4, 112
    torch.manual_seed(11)
    x = torch.randn(n, c, hw, hw, device=DEV).contiguous(memory_format=torch.channels_last)
    gate = torch.rand(n, c, device=DEV)
    res = []
    for fixed in ("1", "0"):
        monkeypatch.setenv("TQ_AEA_FIXED", fixed)
        codes = torch.full((n, hw, hw, cp), 77, dtype=torch.float16, device=DEV)
        out = torch.empty_like(x)
        tq_native.act_encode_act(x, 0.05, 9, 3, codes, act="swish", gate=gate, out=out)
        res.append((codes.float().cpu(), out.view(torch.int32).cpu()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert (res[0][0] != 77).all()


def test_fused_resnet_specialised_epilogues_bit_identical(monkeypatch):
    """The engines' epilogues specialised to the executor's ReLU + code-table form (direct
    engine emit4_relu_lut, TQ_EPI_FAST) give the generic epilogue's bits: every captured conv
    output and code, and the logits."""
    torch.manual_seed(2)
    model = cnn_models.resnet18(pretrained=False).to(DEV).eval()
    settings = cnn_models.static_conv_layer_settings(model, 9, 8, 12)
    q = cnn_models.convert_model(model, settings, 9, 3).to(memory_format=torch.channels_last)
    x = torch.randn(4, 3, 224, 224, device=DEV).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        q(x)
    tr_layer.set_tr_tracking(q, False)
    fused = tq_fuse.FusedResNet(q)
    runs = []
    for fast in ("1", "0"):
        monkeypatch.setenv("TQ_EPI_FAST", fast)
        with torch.no_grad():
            logits = fused(x)  # (bench mode: no fp32 outputs the executor does not need)
        torch.cuda.synchronize()
        runs.append(logits.view(torch.int32).cpu())
    assert torch.equal(runs[0], runs[1])


@pytest.mark.parametrize("seed", range(16))
def test_act_encode_act_random_sweep(seed):
    """Seeded random gate-and-encode passes (tq_act_encode_act): shapes (ragged channel
    chunks, pad channels, non-square maps), activation (none / ReLU / ReLU6 / swish), gate,
    code format and TR settings.  The fp32 output equals torch's composition on the GPU bit
    for bit and the codes are the oracle's TR of (gate x) that value."""
    rng = np.random.default_rng(6000 + seed)
    n, c = int(rng.integers(1, 5)), int(rng.integers(1, 300))
    h, w = int(rng.integers(1, 30)), int(rng.integers(1, 30))
    cp = (c + 7) // 8 * 8 + 8 * int(rng.integers(0, 2))
    act = [None, True, 6, "swish"][int(rng.integers(0, 4))]
    gated = bool(rng.random() < 0.5)
    fmt = torch.float16 if rng.random() < 0.5 else torch.int16
    bw = int(rng.integers(4, 12))
    dt = int(rng.integers(1, 5))
    sf = float(10.0 ** rng.uniform(-3, 0))
    torch.manual_seed(6000 + seed)
    x = (torch.randn(n, c, h, w, device=DEV) * float(10.0 ** rng.uniform(-1, 1.5))).contiguous(
        memory_format=torch.channels_last)
    gate = torch.rand(n, c, device=DEV) if gated else None
    codes = torch.full((n, h, w, cp), 77, dtype=fmt, device=DEV)
    out = torch.empty_like(x)
    tq_native.act_encode_act(x, sf, bw, dt, codes, act=act, gate=gate, out=out)
    if act is None:
        ref = x
    elif act is True:
        ref = torch.relu(x)
    elif act == 6:
        ref = torch.clamp(x, 0.0, 6.0)
    else:
        ref = x * torch.sigmoid(x)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), ref.contiguous(
        memory_format=torch.channels_last).view(torch.int32))
    v = out.permute(0, 2, 3, 1).contiguous()
    if gated:
        v = v * gate[:, None, None, :]
    exp = torch.from_numpy(oracle.tr(v.cpu().numpy(), sf, bw, 1, dt)) / np.float32(sf)
    got = codes.float().cpu()
    assert torch.equal(got[..., :c], exp.round())
    assert (got[..., c:] == 0).all()
