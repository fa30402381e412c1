"""GPU parity of the Cout-64 pixel-ring engine (csrc/tr_conv_c64.hip, MFMA config 15).

The engine sums the same exact integers as every other term-pair engine, so its outputs and
emitted codes must be bit-identical to the VALU engine's (int16 codes, int32 sums, no fp32
windows) on every shape and epilogue form it accepts: the ResNet-18 layer-1 convs (conv1:
ReLU + codes; conv2: + residual, with and without the fp32 output; one or two code outputs),
images smaller and larger than a tile (tiles crossing image boundaries, the widest halo W =
63), every exactness-window setting, and few persistent workgroups (TQ_C64_GRID) so one
workgroup walks many tiles through its pixel ring -- including a partial last tile."""
import pytest
import torch
import torch.nn as nn

import tq_native
import tq_ops
import tr_layer

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
C64 = 15  # MFMA config number of the Cout-64 pixel-ring engine


def _run(codes, lay, hw, *, cfg, sc, sh, res=None, out=True, codes_a=True, codes_b=False,
         fmt=torch.float16, kc_steps=0):
    n = codes.shape[0]
    o = torch.full((n, 64, hw, hw), float("nan"), device=DEV).contiguous(
        memory_format=torch.channels_last) if out else None
    ca = torch.full((n, hw, hw, 64), 7, dtype=torch.int16, device=DEV).to(fmt) \
        if codes_a else None
    cb = torch.full((n, hw, hw, 64), 7, dtype=torch.int16, device=DEV).to(fmt) \
        if codes_b else None
    tq_native.conv2d_termpair_fused(codes, lay.w_codes, 64, 3, 3, (1, 1), (1, 1), (1, 1),
                                    hw, hw, out=o, ch_scale=sc, ch_shift=sh, residual=res,
                                    relu=True, codes_a=ca,
                                    quant_a=(0.05, 9, 3) if codes_a else None, codes_b=cb,
                                    quant_b=(0.11, 9, 2) if codes_b else None, config=cfg,
                                    kc_steps=kc_steps, kc_chunk=-1)
    torch.cuda.synchronize()
    return (None if o is None else o.view(torch.int32).cpu(),
            None if ca is None else ca.float().cpu(),
            None if cb is None else cb.float().cpu())


def _case(hw, batch, seed):
    torch.manual_seed(seed)
    conv = nn.Conv2d(64, 64, 3, 1, 1, bias=False).to(DEV)
    nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
    x = torch.relu(torch.randn(batch, 64, hw, hw, device=DEV)).to(
        memory_format=torch.channels_last)
    sc = (torch.rand(64, dtype=torch.float64, device=DEV) + 0.5) * 2e-4
    sh = torch.randn(64, dtype=torch.float64, device=DEV) * 0.1
    res = torch.randn(batch, 64, hw, hw, device=DEV).contiguous(
        memory_format=torch.channels_last)
    return conv, x, sc, sh, res


def _layers(conv, x, monkeypatch):
    monkeypatch.setenv("TQ_CONV_ENGINE", "valu")
    lay_v = tr_layer.TRConv2dLayer(conv, 9, 3, 9, 8, 12)
    cv = torch.empty((x.shape[0], x.shape[2], x.shape[3], 64), dtype=torch.int16, device=DEV)
    tq_native.act_encode(x, True, 0.02, 9, 3, cv)
    monkeypatch.setenv("TQ_CONV_ENGINE", "mfma")
    lay_m = tr_layer.TRConv2dLayer(conv, 9, 3, 9, 8, 12)
    assert lay_m.engine == "mfma"
    cm = torch.empty_like(cv, dtype=torch.float16)
    tq_native.act_encode(x, True, 0.02, 9, 3, cm)
    return lay_v, cv, lay_m, cm


FORMS = {
    "conv1": dict(out=False),                         # ReLU + codes (block conv1s)
    "conv2_out": dict(res=True),                      # + residual + fp32 out (layer1.0.conv2)
    "conv2_codes": dict(res=True, out=False),         # + residual, codes only (layer1.1.conv2)
    "two_codes": dict(res=True, codes_b=True),        # a second code output
    "out_only": dict(res=True, codes_a=False),        # fp32 output, no codes
}


@pytest.mark.parametrize("hw,batch", [
    (56, 2),    # ResNet-18 layer 1 (12.25 tiles per image: tiles cross images)
    (63, 32),   # the widest halo (W + 1 = 64)
    (20, 8),    # images smaller than a tile: one tile spans 1.6 images
    (7, 32),    # 49-pixel images
])
@pytest.mark.parametrize("grid", ["0", "3", "1"])
def test_c64_bit_identical_to_valu(hw, batch, grid, monkeypatch):
    conv, x, sc, sh, res = _case(hw, batch, seed=hw + batch)
    lay_v, cv, lay_m, cm = _layers(conv, x, monkeypatch)
    monkeypatch.setenv("TQ_C64_GRID", grid)
    for form, kw in FORMS.items():
        kw = dict(kw)
        if kw.pop("res", False):
            kw["res"] = res
        ref = _run(cv, lay_v, hw, cfg=0, sc=sc, sh=sh, fmt=torch.int16, **kw)
        if ref[0] is not None:
            assert not torch.isnan(ref[0].view(torch.float32)).any()
        for kc in (lay_m.kc_steps, lay_m.kc_steps_nonneg, 5, 2, 1):
            got = _run(cm, lay_m, hw, cfg=C64, sc=sc, sh=sh, kc_steps=kc, **kw)
            for g, r in zip(got, ref):
                assert (g is None and r is None) or torch.equal(g, r), (form, kc)


def test_c64_partial_last_tile(monkeypatch):
    """N*H*W = 3 * 56^2 = 9408 = 36.75 tiles: the last tile's upper 64 pixels (two waves'
    blocks) lie past the tensor; the waves that would own them return before their epilogue
    (tr_conv_c64.hip), so the outputs are the VALU engine's bits (the guard tail behind every
    buffer: test_c64_partial_last_tile_leaves_guard_untouched)."""
    conv, x, sc, sh, res = _case(56, 3, seed=5)
    lay_v, cv, lay_m, cm = _layers(conv, x, monkeypatch)
    ref = _run(cv, lay_v, 56, cfg=0, sc=sc, sh=sh, res=res, fmt=torch.int16)
    for grid in ("0", "2", "37"):
        monkeypatch.setenv("TQ_C64_GRID", grid)
        got = _run(cm, lay_m, 56, cfg=C64, sc=sc, sh=sh, res=res, kc_steps=lay_m.kc_steps)
        assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]), grid


def test_c64_is_the_layer1_default(monkeypatch):
    """With no config the dispatcher picks the engine for the layer-1 forms (and TQ_C64=0
    turns it off): same bits either way."""
    conv, x, sc, sh, res = _case(56, 2, seed=9)
    lay_v, cv, lay_m, cm = _layers(conv, x, monkeypatch)
    ref = _run(cv, lay_v, 56, cfg=0, sc=sc, sh=sh, res=res, fmt=torch.int16)
    for flag in ("1", "0"):
        monkeypatch.setenv("TQ_C64", flag)
        got = _run(cm, lay_m, 56, cfg=0, sc=sc, sh=sh, res=res, kc_steps=lay_m.kc_steps)
        assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]), flag


def test_c64_ineligible_shapes_fall_back(monkeypatch):
    """Forms and shapes the engine does not take (N*H*W % 32 != 0, no ReLU, a stride) run the
    default engine under config 15, with the same bits as the VALU engine."""
    conv, x, sc, sh, res = _case(9, 3, seed=13)  # 243 pixels
    lay_v, cv, lay_m, cm = _layers(conv, x, monkeypatch)
    ref = _run(cv, lay_v, 9, cfg=0, sc=sc, sh=sh, res=res, fmt=torch.int16)
    got = _run(cm, lay_m, 9, cfg=C64, sc=sc, sh=sh, res=res, kc_steps=lay_m.kc_steps)
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])


@pytest.mark.parametrize("batch", [64, 256])
def test_c64_bench_size_default_grid(batch, monkeypatch):
    """At the sizes the executor launches it (a 64- or 128-image chunk, the 256-image batch)
    with the default grid -- one workgroup per CU, each walking its share of the 32-pixel
    blocks (ranges of 24.5 / 98 blocks: partial last tiles) -- every form is the VALU
    engine's bits."""
    conv, x, sc, sh, res = _case(56, batch, seed=batch)
    lay_v, cv, lay_m, cm = _layers(conv, x, monkeypatch)
    for form in ("conv1", "conv2_out", "conv2_codes"):
        kw = dict(FORMS[form])
        if kw.pop("res", False):
            kw["res"] = res
        ref = _run(cv, lay_v, 56, cfg=0, sc=sc, sh=sh, fmt=torch.int16, **kw)
        got = _run(cm, lay_m, 56, cfg=C64, sc=sc, sh=sh, kc_steps=lay_m.kc_steps_nonneg, **kw)
        for g, r in zip(got, ref):
            assert (g is None and r is None) or torch.equal(g, r), form


@pytest.mark.parametrize("seed", range(8))
def test_c64_random_sweep(seed, monkeypatch):
    """Seeded random layer-1 engine cases (maps 3-63 -- the widest halo the engine takes --,
    persistent grids of 1 / 2 / 3 / 37 / default workgroups, every epilogue form), the batch
    drawn so that N*H*W is a multiple of the engine's 32-pixel block (the shapes it takes):
    bit-identical to the VALU engine.  TQ_CONFIG_STRICT=1 makes config 15 fail instead of
    falling back to the default engine, so every case runs the c64 engine itself."""
    import math
    import numpy as np
    rng = np.random.default_rng(8000 + seed)
    hw = int(rng.integers(3, 64))
    unit = 32 // math.gcd(hw * hw, 32)
    batch = unit * int(rng.integers(1, max(2, 12 // unit + 1)))
    conv, x, sc, sh, res = _case(hw, batch, seed=8000 + seed)
    lay_v, cv, lay_m, cm = _layers(conv, x, monkeypatch)
    monkeypatch.setenv("TQ_CONFIG_STRICT", "1")
    monkeypatch.setenv("TQ_C64_GRID", str(int(rng.choice([0, 1, 2, 3, 37]))))
    form = sorted(FORMS)[int(rng.integers(0, len(FORMS)))]
    kw = dict(FORMS[form])
    if kw.pop("res", False):
        kw["res"] = res
    ref = _run(cv, lay_v, hw, cfg=0, sc=sc, sh=sh, fmt=torch.int16, **kw)
    got = _run(cm, lay_m, hw, cfg=C64, sc=sc, sh=sh, kc_steps=lay_m.kc_steps, **kw)
    for g, r in zip(got, ref):
        assert (g is None and r is None) or torch.equal(g, r), form


def test_c64_strict_mode_rejects_an_ineligible_shape(monkeypatch):
    """The dispatch probe behind the random sweep: with TQ_CONFIG_STRICT=1 config 15 on a
    shape the engine cannot take (N*H*W = 9 * 9 = 81, not a multiple of 32) is an error, and
    without it the conv quietly runs the default engine."""
    conv, x, sc, sh, res = _case(9, 1, seed=3)
    lay_v, cv, lay_m, cm = _layers(conv, x, monkeypatch)
    ref = _run(cv, lay_v, 9, cfg=0, sc=sc, sh=sh, fmt=torch.int16)
    got = _run(cm, lay_m, 9, cfg=C64, sc=sc, sh=sh, kc_steps=lay_m.kc_steps)
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
    monkeypatch.setenv("TQ_CONFIG_STRICT", "1")
    with pytest.raises(RuntimeError):
        _run(cm, lay_m, 9, cfg=C64, sc=sc, sh=sh, kc_steps=lay_m.kc_steps)


def test_c64_partial_last_tile_leaves_guard_untouched(monkeypatch):
    """Output buffers with a 64 KB guard tail behind the tensor (fp32 output, both code
    outputs) on the partial-last-tile shape: every grid writes exactly the tensor."""
    conv, x, sc, sh, res = _case(56, 3, seed=5)
    lay_v, cv, lay_m, cm = _layers(conv, x, monkeypatch)
    ref = _run(cv, lay_v, 56, cfg=0, sc=sc, sh=sh, res=res, fmt=torch.int16, codes_b=True)
    n, hw, g = 3, 56, 16384
    monkeypatch.setenv("TQ_CONFIG_STRICT", "1")
    for grid in ("0", "2", "37"):
        monkeypatch.setenv("TQ_C64_GRID", grid)
        ob = torch.full((n * hw * hw * 64 + g,), float("nan"), device=DEV)
        o = ob[:n * hw * hw * 64].view(n, hw, hw, 64).permute(0, 3, 1, 2)
        cab = torch.full((n * hw * hw * 64 + g,), 7, dtype=torch.int16, device=DEV).to(
            torch.float16)
        cbb = cab.clone()
        ca = cab[:n * hw * hw * 64].view(n, hw, hw, 64)
        cb = cbb[:n * hw * hw * 64].view(n, hw, hw, 64)
        tq_native.conv2d_termpair_fused(cm, lay_m.w_codes, 64, 3, 3, (1, 1), (1, 1), (1, 1),
                                        hw, hw, out=o, ch_scale=sc, ch_shift=sh, residual=res,
                                        relu=True, codes_a=ca, quant_a=(0.05, 9, 3),
                                        codes_b=cb, quant_b=(0.11, 9, 2), config=C64,
                                        kc_steps=lay_m.kc_steps, kc_chunk=-1)
        torch.cuda.synchronize()
        assert torch.equal(o.contiguous(memory_format=torch.channels_last).view(torch.int32)
                           .cpu(), ref[0]), grid
        assert torch.equal(ca.float().cpu(), ref[1]) and torch.equal(cb.float().cpu(),
                                                                      ref[2]), grid
        assert bool(torch.isnan(ob[n * hw * hw * 64:]).all()), grid
        assert bool((cab[n * hw * hw * 64:] == 7).all()) and bool(
            (cbb[n * hw * hw * 64:] == 7).all()), grid


@pytest.mark.parametrize("form", ["conv1", "conv2_out", "conv2_codes"])
def test_epi_fast_off_routes_layer1_forms_bit_identically(form, monkeypatch):
    """TQ_EPI_FAST=0 (the generic-epilogue A/B switch) turns the c64 default off for the
    layer-1 forms and the ring engine's forms over to the generic epilogue; the bits stay the
    VALU engine's."""
    conv, x, sc, sh, res = _case(28, 4, seed=21)
    lay_v, cv, lay_m, cm = _layers(conv, x, monkeypatch)
    kw = dict(FORMS[form])
    if kw.pop("res", False):
        kw["res"] = res
    ref = _run(cv, lay_v, 28, cfg=0, sc=sc, sh=sh, fmt=torch.int16, **kw)
    monkeypatch.setenv("TQ_EPI_FAST", "0")
    for ring in ("0", "1"):
        monkeypatch.setenv("TQ_RING", ring)
        got = _run(cm, lay_m, 28, cfg=0, sc=sc, sh=sh, kc_steps=lay_m.kc_steps, **kw)
        for gg, r in zip(got, ref):
            assert (gg is None and r is None) or torch.equal(gg, r), (form, ring)
