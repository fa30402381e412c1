"""GPU parity of the expand engine (csrc/tr_conv_xp.hip, MFMA config 14).

The engine sums the same exact integers as every other term-pair engine and runs the shared
epilogue, so its outputs and emitted codes must be bit-identical to the VALU engine's (int16
codes, int32 sums; for swish, which only the MFMA engines' epilogue has, the direct engine's)
on every shape it accepts: MobileNet-V2 / EfficientNet-b0 expand shapes
(input channels not a multiple of 64, one and two K-steps), partial Cout tiles, every
epilogue form the fused executors use (ReLU6 codes, swish with the fp32 output, two code
outputs, signed codes), layers split into Cout groups, and few persistent workgroups per
group (TQ_XP_GRID) so each wave walks many pixel tiles."""
import pytest
import torch
import torch.nn as nn

import tq_native
import tq_ops
import tr_layer

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
XP = 14  # MFMA config number of the expand engine
DIRECT = 10  # the direct engine, 64-row Cout tiles (bit-identical to the VALU engine)


def _layers(cin, cout, monkeypatch, seed):
    torch.manual_seed(seed)
    conv = nn.Conv2d(cin, cout, 1, 1, 0, bias=False).to(DEV)
    nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
    monkeypatch.setenv("TQ_CONV_ENGINE", "valu")
    lay_v = tr_layer.TRConv2dLayer(conv, 9, 3, 9, 8, 12)
    monkeypatch.setenv("TQ_CONV_ENGINE", "mfma")
    lay_m = tr_layer.TRConv2dLayer(conv, 9, 3, 9, 8, 12)
    assert lay_m.engine == "mfma"
    return lay_v, lay_m


def _run(x, lay, cout, hw, *, cfg, sc, sh, fmt, act, out, codes_b, kc_steps=0):
    n = x.shape[0]
    cp_in = tq_ops.act_channels(x.shape[1])
    codes = torch.empty((n, hw, hw, cp_in), dtype=torch.int16, device=DEV).to(fmt)
    tq_native.act_encode(x, True, 0.02, 9, 3, codes)
    o = torch.full((n, cout, hw, hw), float("nan"), device=DEV).contiguous(
        memory_format=torch.channels_last) if out else None
    cpo = tq_ops.act_channels(cout)
    ca = torch.full((n, hw, hw, cpo), 7, dtype=torch.int16, device=DEV).to(torch.float16)
    cb = torch.full((n, hw, hw, cpo), 7, dtype=torch.int16, device=DEV).to(torch.float16) \
        if codes_b else None
    tq_native.conv2d_termpair_fused(codes, lay.w_codes, cout, 1, 1, (1, 1), (0, 0), (1, 1),
                                    hw, hw, out=o, ch_scale=sc, ch_shift=sh, relu=act,
                                    codes_a=ca, quant_a=(0.05, 9, 3), codes_b=cb,
                                    quant_b=(0.11, 9, 2) if codes_b else None, config=cfg,
                                    kc_steps=kc_steps)
    torch.cuda.synchronize()
    return (None if o is None else o.view(torch.int32).cpu(), ca.float().cpu(),
            None if cb is None else cb.float().cpu())


@pytest.mark.parametrize("cin,cout,hw,batch", [
    (16, 96, 28, 3),     # MobileNet-V2 block 2 expand (Cp 16: one K-step, 48 zero codes)
    (24, 144, 14, 5),    # three Cout tiles, the last one 16 rows
    (40, 240, 9, 7),     # EfficientNet-b0 (P not a multiple of 32)
    (64, 256, 7, 6),     # four Cout tiles (32 KB of weights: one Cout group)
    (96, 100, 7, 3),     # two K-steps, partial Cout tile, pad code channels (cp 104)
    (64, 384, 7, 4),     # two Cout groups of four tiles
    (96, 576, 7, 3),     # two K-steps: five Cout groups of two tiles, the last one of one
])
@pytest.mark.parametrize("form", ["relu6_codes", "relu_codes", "swish_codes", "swish_out",
                                  "two_codes", "signed"])
@pytest.mark.parametrize("grid", ["0", "3"])
def test_xp_bit_identical_to_valu(cin, cout, hw, batch, form, grid, monkeypatch):
    lay_v, lay_m = _layers(cin, cout, monkeypatch, seed=cin + cout)
    x = torch.relu(torch.randn(batch, cin, hw, hw, device=DEV)).contiguous(
        memory_format=torch.channels_last)
    sc = (torch.rand(cout, dtype=torch.float64, device=DEV) + 0.5) * 2e-4
    sh = torch.randn(cout, dtype=torch.float64, device=DEV) * 0.1
    kw = dict(relu6_codes=dict(act=6, out=False, codes_b=False),   # (the specialised forms)
              relu_codes=dict(act=True, out=False, codes_b=False),
              swish_codes=dict(act="swish", out=False, codes_b=False),
              swish_out=dict(act="swish", out=True, codes_b=False),
              two_codes=dict(act=True, out=True, codes_b=True),
              signed=dict(act=False, out=True, codes_b=False))[form]
    if form.startswith("swish"):  # (the swish epilogue exists on the MFMA direct engine only)
        ref = _run(x, lay_m, cout, hw, cfg=DIRECT, sc=sc, sh=sh, fmt=torch.float16,
                   kc_steps=lay_m.kc_steps, **kw)
    else:
        ref = _run(x, lay_v, cout, hw, cfg=0, sc=sc, sh=sh, fmt=torch.int16, **kw)
    monkeypatch.setenv("TQ_XP_GRID", grid)
    monkeypatch.setenv("TQ_XP_GROUPS", "8")  # (the wide shapes: Cout groups)
    got = _run(x, lay_m, cout, hw, cfg=XP, sc=sc, sh=sh, fmt=torch.float16,
               kc_steps=lay_m.kc_steps, **kw)
    for g, r in zip(got, ref):
        assert (g is None and r is None) or torch.equal(g, r)


def test_xp_default_switch(monkeypatch):
    """The heuristic (config 0) routes eligible 1x1 convs through the engine by default and
    TQ_XP=0 through the direct engine: the same bits either way."""
    lay_v, lay_m = _layers(16, 96, monkeypatch, seed=5)
    x = torch.relu(torch.randn(2, 16, 14, 14, device=DEV)).contiguous(
        memory_format=torch.channels_last)
    sc = torch.full((96,), 1e-4, dtype=torch.float64, device=DEV)
    sh = torch.zeros(96, dtype=torch.float64, device=DEV)
    ref = _run(x, lay_v, 96, 14, cfg=0, sc=sc, sh=sh, fmt=torch.int16, act=6, out=True,
               codes_b=False)
    for v in ("1", "0"):
        monkeypatch.setenv("TQ_XP", v)
        got = _run(x, lay_m, 96, 14, cfg=0, sc=sc, sh=sh, fmt=torch.float16, act=6, out=True,
                   codes_b=False, kc_steps=lay_m.kc_steps)
        assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]), v


@pytest.mark.parametrize("seed", range(12))
def test_xp_random_sweep(seed, monkeypatch):
    """Seeded random expand-engine cases (input channels 8-96, Cout a multiple of 4 up to 600,
    maps 3-30, batch 1-8, persistent grids, every epilogue form): bit-identical to the VALU
    engine (swish: to the direct engine, the other MFMA engine with that epilogue)."""
    import numpy as np
    rng = np.random.default_rng(9000 + seed)
    cin = 8 * int(rng.integers(1, 13))
    cout = 4 * int(rng.integers(2, 151))
    hw = int(rng.integers(3, 31))
    batch = int(rng.integers(1, 9))
    form = ["relu6_codes", "relu_codes", "swish_codes", "swish_out", "two_codes",
            "signed"][int(rng.integers(0, 6))]
    lay_v, lay_m = _layers(cin, cout, monkeypatch, seed=9000 + seed)
    x = torch.relu(torch.randn(batch, cin, hw, hw, device=DEV)).contiguous(
        memory_format=torch.channels_last)
    sc = (torch.rand(cout, dtype=torch.float64, device=DEV) + 0.5) * 2e-4
    sh = torch.randn(cout, dtype=torch.float64, device=DEV) * 0.1
    kw = dict(relu6_codes=dict(act=6, out=False, codes_b=False),
              relu_codes=dict(act=True, out=False, codes_b=False),
              swish_codes=dict(act="swish", out=False, codes_b=False),
              swish_out=dict(act="swish", out=True, codes_b=False),
              two_codes=dict(act=True, out=True, codes_b=True),
              signed=dict(act=False, out=True, codes_b=False))[form]
    if form.startswith("swish"):
        ref = _run(x, lay_m, cout, hw, cfg=DIRECT, sc=sc, sh=sh, fmt=torch.float16,
                   kc_steps=lay_m.kc_steps, **kw)
    else:
        ref = _run(x, lay_v, cout, hw, cfg=0, sc=sc, sh=sh, fmt=torch.int16, **kw)
    monkeypatch.setenv("TQ_XP_GRID", str(int(rng.choice([0, 1, 3]))))
    monkeypatch.setenv("TQ_XP_GROUPS", "8")
    got = _run(x, lay_m, cout, hw, cfg=XP, sc=sc, sh=sh, fmt=torch.float16,
               kc_steps=lay_m.kc_steps, **kw)
    for g, r in zip(got, ref):
        assert (g is None and r is None) or torch.equal(g, r), form
