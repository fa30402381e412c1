"""GPU parity of the tap-ring engine (csrc/tr_conv_ring.hip, MFMA config 13).

The engine sums the same exact integers as every other term-pair engine, so its outputs and
emitted codes must be bit-identical to the VALU engine's (int16 codes, int32 sums, no fp32
windows at all) on every shape it accepts: ResNet-18's layer-2/3/4 3x3 convs and odd ones
(tiles crossing image boundaries, partial Cout tiles, one and three channel chunks), with
every epilogue form the fused executor uses, the chunk-major exactness windows, and few
persistent workgroups (TQ_RING_GRID) so each one walks many tiles -- the path where the weight
ring and the patch stream run across tile boundaries."""
import pytest
import torch
import torch.nn as nn

import tq_native
import tq_ops
import tr_layer

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
RING = 13  # MFMA config number of the tap-ring engine


@pytest.fixture(autouse=True, params=["1", "2"])
def shape(request, monkeypatch):
    """Both engine shapes: 1 = one 8-wave workgroup per CU (128 x 256 tiles, 64-code K-steps),
    2 = two 4-wave workgroups per CU (128 x 128 tiles, 32-code K-steps)."""
    monkeypatch.setenv("TQ_RING_V", request.param)
    return request.param


def _run(codes, lay, cout, hw, *, cfg, sc, sh, res=None, relu=True, out=True, codes_b=False,
         fmt=torch.float16, kc_steps=0, kc_chunk=-1, codes_a=True):
    n = codes.shape[0]
    o = torch.full((n, cout, hw, hw), float("nan"), device=DEV).contiguous(
        memory_format=torch.channels_last) if out else None
    cpo = tq_ops.act_channels(cout)
    ca = torch.full((n, hw, hw, cpo), 7, dtype=torch.int16, device=DEV).to(fmt) \
        if codes_a else None
    cb = torch.full((n, hw, hw, cpo), 7, dtype=torch.int16, device=DEV).to(fmt) \
        if codes_b else None
    tq_native.conv2d_termpair_fused(codes, lay.w_codes, cout, 3, 3, (1, 1), (1, 1), (1, 1),
                                    hw, hw, out=o, ch_scale=sc, ch_shift=sh, residual=res,
                                    relu=relu, codes_a=ca,
                                    quant_a=(0.05, 9, 3) if codes_a else None, codes_b=cb,
                                    quant_b=(0.11, 9, 2) if codes_b else None, config=cfg,
                                    kc_steps=kc_steps, kc_chunk=kc_chunk)
    torch.cuda.synchronize()
    return (None if o is None else o.view(torch.int32).cpu(),
            None if ca is None else ca.float().cpu(),
            None if cb is None else cb.float().cpu())


def _case(cin, cout, hw, batch, seed):
    torch.manual_seed(seed)
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=False).to(DEV)
    nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
    x = torch.relu(torch.randn(batch, cin, hw, hw, device=DEV)).to(
        memory_format=torch.channels_last)
    sc = (torch.rand(cout, dtype=torch.float64, device=DEV) + 0.5) * 2e-4
    sh = torch.randn(cout, dtype=torch.float64, device=DEV) * 0.1
    res = torch.randn(batch, cout, hw, hw, device=DEV).contiguous(
        memory_format=torch.channels_last)
    return conv, x, sc, sh, res


def _layers(conv, x, monkeypatch):
    cp = tq_ops.act_channels(conv.in_channels)
    monkeypatch.setenv("TQ_CONV_ENGINE", "valu")
    lay_v = tr_layer.TRConv2dLayer(conv, 9, 3, 9, 8, 12)
    cv = torch.empty((x.shape[0], x.shape[2], x.shape[3], cp), dtype=torch.int16, device=DEV)
    tq_native.act_encode(x, True, 0.02, 9, 3, cv)
    monkeypatch.setenv("TQ_CONV_ENGINE", "mfma")
    lay_m = tr_layer.TRConv2dLayer(conv, 9, 3, 9, 8, 12)
    assert lay_m.engine == "mfma"
    cm = torch.empty_like(cv, dtype=torch.float16)
    tq_native.act_encode(x, True, 0.02, 9, 3, cm)
    return lay_v, cv, lay_m, cm


@pytest.mark.parametrize("cin,cout,hw,batch", [
    (128, 128, 28, 5),    # layer 2: R = 9 rows per tile, tiles cross images
    (256, 256, 14, 6),    # layer 3: two Cout tiles per pixel tile
    (512, 512, 7, 9),     # layer 4: 36-row tiles over 5 images
    (64, 64, 56, 2),      # layer 1 shape (one chunk, half-empty Cout tile)
    (192, 132, 9, 3),     # three chunks, partial Cout tile, R = 28; with one workgroup
                          # its second tile starts at ring slot 27 mod NR != 0
])
@pytest.mark.parametrize("grid", ["0", "3", "1"])
def test_ring_bit_identical_to_valu(cin, cout, hw, batch, grid, monkeypatch):
    conv, x, sc, sh, res = _case(cin, cout, hw, batch, seed=cin + cout + hw)
    lay_v, cv, lay_m, cm = _layers(conv, x, monkeypatch)
    ref = _run(cv, lay_v, cout, hw, cfg=0, sc=sc, sh=sh, res=res, codes_b=True,
               fmt=torch.int16)
    assert not torch.isnan(ref[0].view(torch.float32)).any()
    monkeypatch.setenv("TQ_RING_GRID", grid)
    for kc in ((lay_m.kc_steps, lay_m.kc_chunk), (lay_m.kc_steps_nonneg, lay_m.kc_chunk_nonneg),
               (5, 2), (1, 1)):
        got = _run(cm, lay_m, cout, hw, cfg=RING, sc=sc, sh=sh, res=res, codes_b=True,
                   kc_steps=kc[0], kc_chunk=kc[1])
        assert torch.equal(got[0], ref[0]), kc
        assert torch.equal(got[1], ref[1]) and torch.equal(got[2], ref[2]), kc


@pytest.mark.parametrize("form", ["codes_only", "no_relu", "out_only", "last_conv",
                                  "last_conv_generic"])
def test_ring_epilogue_forms(form, monkeypatch):
    """The fused executor's other epilogue forms: codes only (no fp32 output, no residual),
    signed values (no ReLU: code tables negated), fp32 output without codes_b, and the last
    conv's ReLU + residual + fp32 output with no codes (specialised form 2; TQ_EPI_FAST=0
    the generic epilogue)."""
    conv, x, sc, sh, res = _case(256, 256, 14, 4, seed=3)
    lay_v, cv, lay_m, cm = _layers(conv, x, monkeypatch)
    kw = dict(codes_only=dict(out=False), no_relu=dict(relu=False, res=res),
              out_only=dict(res=res), last_conv=dict(res=res, codes_a=False),
              last_conv_generic=dict(res=res, codes_a=False))[form]
    if form == "last_conv_generic":
        monkeypatch.setenv("TQ_EPI_FAST", "0")
    ref = _run(cv, lay_v, 256, 14, cfg=0, sc=sc, sh=sh, fmt=torch.int16, **kw)
    monkeypatch.setenv("TQ_RING_GRID", "5")
    got = _run(cm, lay_m, 256, 14, cfg=RING, sc=sc, sh=sh, kc_steps=lay_m.kc_steps,
               kc_chunk=lay_m.kc_chunk, **kw)
    for g, r in zip(got, ref):
        assert (g is None and r is None) or torch.equal(g, r)


def test_ring_m_slow_order(monkeypatch):
    """Cout-tile-major tile order (TQ_MSLOW=1) walks the same tiles in another order."""
    conv, x, sc, sh, res = _case(256, 512, 7, 7, seed=11)
    lay_v, cv, lay_m, cm = _layers(conv, x, monkeypatch)
    ref = _run(cv, lay_v, 512, 7, cfg=0, sc=sc, sh=sh, res=res, fmt=torch.int16)
    monkeypatch.setenv("TQ_RING_GRID", "4")
    monkeypatch.setenv("TQ_MSLOW", "1")
    got = _run(cm, lay_m, 512, 7, cfg=RING, sc=sc, sh=sh, res=res, kc_steps=lay_m.kc_steps,
               kc_chunk=lay_m.kc_chunk)
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])


@pytest.mark.parametrize("cin,cout,hw,batch", [
    (128, 128, 28, 5),    # 2 chunks per tile
    (256, 256, 14, 6),    # 4 chunks, two Cout tiles
    (512, 512, 7, 9),     # 8 chunks, four Cout tiles: with 37 workgroups a tile spans up to 6
    (192, 132, 9, 3),     # 3 chunks, partial Cout tile
])
@pytest.mark.parametrize("grid", ["0", "3", "7", "37"])
def test_ring_stream_k_bit_identical(cin, cout, hw, batch, grid, shape, monkeypatch):
    """Stream-K split (TQ_RING_SK=2 forces it wherever it applies): tiles split at chunk
    boundaries over 2..6 workgroups, the last contributor adding the others' int32 slabs --
    the same bits as the VALU engine, with and without int32 exactness windows; every launch
    leaves its tile counters at zero for the next one (the cases share one workspace)."""
    conv, x, sc, sh, res = _case(cin, cout, hw, batch, seed=cin + 7 * cout + hw)
    lay_v, cv, lay_m, cm = _layers(conv, x, monkeypatch)
    ref = _run(cv, lay_v, cout, hw, cfg=0, sc=sc, sh=sh, res=res, codes_b=True,
               fmt=torch.int16)
    monkeypatch.setenv("TQ_RING_GRID", grid)
    monkeypatch.setenv("TQ_RING_SK", "2")
    for kc in ((lay_m.kc_steps, lay_m.kc_chunk), (lay_m.kc_steps_nonneg, lay_m.kc_chunk_nonneg),
               (1, 1)):
        for form in ("res", "codes_only"):
            if form == "res":
                r = ref
                got = _run(cm, lay_m, cout, hw, cfg=RING, sc=sc, sh=sh, res=res, codes_b=True,
                           kc_steps=kc[0], kc_chunk=kc[1])
            else:
                r = _run(cv, lay_v, cout, hw, cfg=0, sc=sc, sh=sh, out=False, fmt=torch.int16)
                got = _run(cm, lay_m, cout, hw, cfg=RING, sc=sc, sh=sh, out=False,
                           kc_steps=kc[0], kc_chunk=kc[1])
            for g, e in zip(got, r):
                assert (g is None and e is None) or torch.equal(g, e), (kc, form)


@pytest.mark.parametrize("seed", range(8))
def test_ring_random_sweep(seed, monkeypatch):
    """Seeded random ring-engine shapes (1-8 channel chunks, Cout a multiple of 4 up to 520,
    maps 3-30, batch 1-8, persistent grids of 1 / 3 / 7 / default workgroups): outputs and
    both code targets bit-identical to the VALU engine's."""
    import numpy as np
    rng = np.random.default_rng(7000 + seed)
    cin = 64 * int(rng.integers(1, 9))
    cout = 4 * int(rng.integers(2, 131))
    hw = int(rng.integers(3, 31))
    batch = int(rng.integers(1, 9))
    conv, x, sc, sh, res = _case(cin, cout, hw, batch, seed=7000 + seed)
    lay_v, cv, lay_m, cm = _layers(conv, x, monkeypatch)
    ref = _run(cv, lay_v, cout, hw, cfg=0, sc=sc, sh=sh, res=res, codes_b=True,
               fmt=torch.int16)
    monkeypatch.setenv("TQ_RING_GRID", str(int(rng.choice([0, 1, 3, 7]))))
    got = _run(cm, lay_m, cout, hw, cfg=RING, sc=sc, sh=sh, res=res, codes_b=True,
               kc_steps=lay_m.kc_steps, kc_chunk=lay_m.kc_chunk)
    assert torch.equal(got[0], ref[0])
    assert torch.equal(got[1], ref[1]) and torch.equal(got[2], ref[2])
