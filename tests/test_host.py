"""Host-side logic on the CPU: model conversion rules, the term-pair MAC / parameter-bit
counter against the reference's published results/*.json, calibration bookkeeping.

TR layers are built on CPU with the TR op replaced by a stand-in (the oracle, or an
identity stub where only shapes matter) so these tests isolate the host logic; the product's
own CPU TR op (libtq_host.so) is tested in test_host_tr.py."""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

import oracle
import tq_ops
import tr_layer
import cnn_models
import profile_model

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PUBLISHED = json.load(open(os.path.join(GOLDEN, "published_results.json")))


def _oracle_tr(input, sf, bitwidth, group_size, num_keep_terms):
    return torch.from_numpy(oracle.tr(input.detach().contiguous().numpy(), sf, bitwidth,
                                      group_size, num_keep_terms))


def _oracle_tr_encode(w, sf, bitwidth, group_size, num_keep_terms):
    out = _oracle_tr(w, sf, bitwidth, group_size, num_keep_terms)
    codes = torch.round(out.double() / float(np.float32(sf))).to(torch.int32)
    return out, codes


def _stub_tr(input, sf, bitwidth, group_size, num_keep_terms):
    return input.detach().clone()


def _stub_tr_encode(w, sf, bitwidth, group_size, num_keep_terms):
    return w.detach().clone(), torch.zeros(w.shape, dtype=torch.int32)


@pytest.fixture
def oracle_tr(monkeypatch):
    monkeypatch.setattr(tq_ops, "tr", _oracle_tr)
    monkeypatch.setattr(tq_ops, "tr_encode", _oracle_tr_encode)


@pytest.fixture
def stub_tr(monkeypatch):
    monkeypatch.setattr(tq_ops, "tr", _stub_tr)
    monkeypatch.setattr(tq_ops, "tr_encode", _stub_tr_encode)


def _tmacs(arch, wb, g, k, db, dt):
    torch.manual_seed(0)
    model = getattr(cnn_models, arch)(pretrained=False).eval()
    settings = cnn_models.static_conv_layer_settings(model, wb, g, k)
    qmodel = cnn_models.convert_model(model, settings, db, dt)
    x = torch.randn(1, 3, 224, 224)
    return profile_model.get_model_ops(qmodel, (x,))


@pytest.mark.parametrize("i,k", list(enumerate([8, 10, 12, 14, 16])))
def test_resnet18_tmacs_match_published(stub_tr, i, k):
    tmacs, _ = _tmacs("resnet18", 9, 8, k, 9, 3)
    assert tmacs == PUBLISHED["resnet18-results.json"]["tr-data3"]["tmacs"][i]
    tmacs2, _ = _tmacs("resnet18", 9, 8, k, 9, 2)
    assert tmacs2 == PUBLISHED["resnet18-results.json"]["tr-data2"]["tmacs"][i]


def test_resnet18_group_size_grid_tmacs(stub_tr):
    pub = PUBLISHED["resnet18-group-size-results.json"]
    for g in [1, 2, 8, 16, 32]:
        for i, avg in enumerate([1.0, 1.25, 1.5, 2.0, 3.0]):
            k = round(avg * g)  # evaluate_group_size.py:81 (banker's rounding)
            tmacs, _ = _tmacs("resnet18", 9, g, k, 9, 3)
            assert tmacs == pub[str(g)]["tmacs"][i], (g, avg)


def test_efficientnet_tmacs_match_published(stub_tr):
    """The hand-built EfficientNet-b0 reproduces the published counts exactly, which pins its
    architecture (layer shapes, and which convs get the (16, 1, 16) setting)."""
    key = "efficientnet_b0-results.json"
    for dt in (2, 3, 4):
        for i, k in enumerate([12, 16, 20, 24]):
            tmacs, _ = _tmacs("efficientnet_b0", 9, 8, k, 9, dt)
            assert tmacs == PUBLISHED[key]["tr-data%d" % dt]["tmacs"][i], (dt, k)


def test_mobilenet_tmacs_match_published(stub_tr):
    """MobileNet-V2's published counts include its 17 depthwise convs (20,716,416 MAC/image,
    counted at alpha = 16/1): they were produced before profile_model.py:25 gained the
    `groups == 1` condition.  The current rule's count plus that depthwise term reproduces
    every published value (fp32-accumulated, so compared at 1e-7)."""
    key = "mobilenet_v2-results.json"
    dw_macs = 20716416
    for dt in (2, 3, 4):
        for i, k in enumerate([12, 16, 20, 24]):
            tmacs, _ = _tmacs("mobilenet_v2", 9, 8, k, 9, dt)
            pub = PUBLISHED[key]["tr-data%d" % dt]["tmacs"][i]
            assert tmacs + dw_macs * 16 * dt == pytest.approx(pub, rel=1e-7), (dt, k)


def test_vgg16_tmacs_match_published(stub_tr):
    for i, k in enumerate([8, 10, 12, 14, 16]):
        tmacs, _ = _tmacs("vgg16_bn", 9, 8, k, 9, 3)
        assert tmacs == PUBLISHED["vgg16_bn-results.json"]["tr-data3"]["tmacs"][i]


def test_avg_terms_match_published():
    import evaluate_cnn
    for arch, key in [("resnet18", "resnet18-results.json"),
                      ("mobilenet_v2", "mobilenet_v2-results.json"),
                      ("efficientnet_b0", "efficientnet_b0-results.json")]:
        model = getattr(cnn_models, arch)(pretrained=False)
        ks = [8, 10, 12, 14, 16] if arch == "resnet18" else [12, 16, 20, 24]
        for i, k in enumerate(ks):
            settings = cnn_models.static_conv_layer_settings(model, 9, 8, k)
            assert evaluate_cnn.compute_avg_terms(settings) == pytest.approx(
                PUBLISHED[key]["tr-data3"]["avg_terms"][i])


def test_replace_conv_layers_rules(stub_tr):
    model = cnn_models.resnet18(pretrained=False)
    settings = cnn_models.static_conv_layer_settings(model, 9, 8, 12)
    assert settings[0] == (16, 1, 16) and all(s == (9, 8, 12) for s in settings[1:])
    assert len(settings) == 20
    q = cnn_models.convert_model(model, settings, 9, 3)
    tr = [n for n, m in q.named_modules() if isinstance(m, tr_layer.TRConv2dLayer)]
    assert len(tr) == 19 and "conv1" not in tr and "layer2.0.downsample.0" in tr
    assert isinstance(q.conv1, nn.Conv2d)
    # the original model is untouched (convert_model deep-copies)
    assert not any(isinstance(m, tr_layer.TRConv2dLayer) for m in model.modules())
    mb = cnn_models.mobilenet_v2(pretrained=False)
    st = cnn_models.static_conv_layer_settings(mb, 9, 8, 12)
    convs = [m for m in mb.modules() if isinstance(m, nn.Conv2d)]
    for c, s in zip(convs, st):
        if c.groups > 1:
            assert s == (16, 1, 16)


def test_trconv_layer_weight_is_reference_tr(oracle_tr):
    torch.manual_seed(1)
    conv = nn.Conv2d(16, 8, 3, padding=1)
    w = conv.weight.detach().clone()
    layer = tr_layer.TRConv2dLayer(conv, 9, 3, 9, 8, 12)
    sf = w.abs().max().item() / 2 ** 8
    assert layer.w_sf == sf
    assert torch.equal(layer.conv.weight.detach(), torch.from_numpy(oracle.tr(w.numpy(), sf, 9,
                                                                              8, 12)))
    # 9-bit codes are exact fp16 values: the MFMA engine (fp16 codes, Kp % 64 == 0)
    assert layer.termpair and layer.engine == "mfma"
    assert layer.w_codes.dtype == torch.float16 and layer.kc_steps == 0
    assert layer.w_codes.shape[1] % 64 == 0 and layer.w_codes.shape[0] % 128 == 0
    # packed codes reproduce the fake-quantized weights: [O][kh][kw][c] order
    packed = layer.w_codes[:8, :9 * 16].view(8, 3, 3, 16).permute(0, 3, 1, 2).float()
    assert torch.equal(packed * np.float32(sf), layer.conv.weight.detach())
    for attr in ("conv", "input_quant", "w_sf", "group_size", "num_terms", "weight_bits",
                 "data_bits", "data_terms"):
        assert hasattr(layer, attr)


def test_trconv_layer_engine_choice(oracle_tr, monkeypatch):
    torch.manual_seed(2)
    conv = nn.Conv2d(16, 8, 3, padding=1)
    lay = tr_layer.TRConv2dLayer(conv, 12, 3, 9, 8, 12)  # 12-bit activations: not fp16-exact
    assert lay.engine == "valu" and lay.w_codes.dtype == torch.int16
    assert lay.w_codes.shape[1] % 32 == 0
    monkeypatch.setenv("TQ_CONV_ENGINE", "valu")
    lay = tr_layer.TRConv2dLayer(nn.Conv2d(16, 8, 3, padding=1), 9, 3, 9, 8, 12)
    assert lay.engine == "valu"
    monkeypatch.setenv("TQ_CONV_ENGINE", "bogus")
    with pytest.raises(RuntimeError, match="TQ_CONV_ENGINE"):
        tr_layer.TRConv2dLayer(nn.Conv2d(16, 8, 3, padding=1), 9, 3, 9, 8, 12)


def test_tracking_histogram_and_passthrough(stub_tr):
    conv = nn.Conv2d(4, 4, 1)
    layer = tr_layer.TRConv2dLayer(conv, 8, 3, 8, 1, 8)
    x = torch.randn(2, 4, 3, 3)
    with torch.no_grad():
        y = layer(x)
    assert torch.allclose(y, conv(x))
    assert layer.input_quant.hist_bins.sum().item() == x.numel()
    assert torch.equal(layer.input_quant.hist_bins, torch.histc(x, 8192, -50, 50))


def test_set_tr_tracking_calls_finish(stub_tr, monkeypatch):
    calls = []
    monkeypatch.setattr(tr_layer, "mse_profile",
                        lambda h, lo, hi, b, t: calls.append((b, t)) or 0.125)
    model = nn.Sequential(nn.Conv2d(3, 4, 1), nn.Conv2d(4, 4, 1))
    model[1] = tr_layer.TRConv2dLayer(model[1], 9, 3, 9, 1, 9)
    tr_layer.set_tr_tracking(model, False)
    assert calls == [(9, 3)]
    assert model[1].input_quant.sf == 0.125 and not model[1].input_quant.tracking
    tr_layer.set_tr_tracking(model, True)
    assert model[1].input_quant.tracking


def test_tr_layer_hese_matches_reference_lengths():
    g = np.load(os.path.join(GOLDEN, "tr_layer_hese_len.npz"))
    got = [len(tr_layer.hese(int(q))) for q in g["q"]]
    assert got == g["length"].tolist()
    lens = tr_layer._hese_len_tensor(torch.from_numpy(g["q"]))
    assert lens.tolist() == g["length"].tolist()
    # value is preserved: the run form sums back to the number
    for q in range(-300, 300):
        assert sum(tr_layer.hese(q)) == q


def test_compute_compressed_hese_matches_python_loop():
    torch.manual_seed(5)
    w = torch.randn(64, 32) * 0.1
    sf = w.abs().max().item() / 8
    bits = tr_layer.compute_compressed_hese(w, sf, 8)
    q = (w / sf).int()
    exp = (int(np.ceil(np.log2(8))) + 2) * sum(oracle.tr_layer_hese_len(v)
                                               for v in q.view(-1).tolist())
    assert bits == exp


def test_mnist_mlp_counts_match_published(stub_tr):
    import evaluate_mlp
    from train_mlp import MNISTMLP
    torch.manual_seed(0)
    x = torch.randn(1, 1, 28, 28)
    pub_q = PUBLISHED["mnist-quant.json"]
    for i, wb in enumerate([2, 3, 4, 5, 6]):  # evaluate_mlp.sh:3 (g=1, wt=wb, db=dt=6)
        m = MNISTMLP()
        st = evaluate_mlp.static_linear_layer_settings(m, wb, 1, wb)
        q = evaluate_mlp.replace_linear_layers(m, st, 6, 6)
        tmacs, bits = profile_model.get_model_ops(q, (x,))
        assert tmacs == pub_q["tmacs"][i] and bits == pub_q["param_bits"][i]
    pub_t = PUBLISHED["mnist-tr.json"]
    for i, wt in enumerate([6, 8, 10, 12, 14]):  # evaluate_mlp.sh:4 (wb=4, g=16, db=dt=6)
        m = MNISTMLP()
        st = evaluate_mlp.static_linear_layer_settings(m, 4, 16, wt)
        q = evaluate_mlp.replace_linear_layers(m, st, 6, 6)
        tmacs, _ = profile_model.get_model_ops(q, (x,))
        assert tmacs == pub_t["tmacs"][i]


def test_lstm_counts_match_published(stub_tr):
    """Decoder-only term-pair MACs of one 35x10 batch and the g=1 parameter bits of the
    LSTM-650 sweeps (evaluate_lstm.sh), fp32-accumulated like thop."""
    import evaluate_lstm
    from lstm_models.model import RNNModel
    torch.manual_seed(0)
    model = RNNModel("LSTM", evaluate_lstm.WT2_VOCAB, 650, 650, 2, 0.5, True)
    data = torch.randint(0, evaluate_lstm.WT2_VOCAB, (35, 10))
    inputs = (data, model.init_hidden(10))
    pub_q = PUBLISHED["lstm-quant.json"]
    for i, wb in enumerate([5, 6, 7, 8, 9]):
        st = evaluate_lstm.static_lstm_layer_settings(model, wb, 1, wb)
        q = evaluate_lstm.convert_model(model, st, 8, 8)
        tmacs, bits = profile_model.get_model_ops(q, inputs)
        assert tmacs == pub_q["tmacs"][i] and bits == pub_q["param_bits"][i]
    pub_t = PUBLISHED["lstm-tr.json"]
    for i, wt in enumerate([8, 12, 16, 20, 24]):
        st = evaluate_lstm.static_lstm_layer_settings(model, 8, 8, wt)
        q = evaluate_lstm.convert_model(model, st, 8, 8)
        tmacs, _ = profile_model.get_model_ops(q, inputs)
        assert tmacs == pub_t["tmacs"][i]


def test_mfma_flush_steps_bounds():
    import tq_ops  # noqa: F811
    codes = torch.full((4, 64, 3, 3), 256, dtype=torch.int32)
    packed, _ = tq_ops.pack_conv_weight(codes, "mfma")
    assert tq_ops.mfma_flush_steps(packed, 9) == 2
    assert tq_ops.mfma_flush_steps(packed, 8) == 4
    assert tq_ops.mfma_flush_steps(packed, 11) == -1
    small = torch.ones((4, 64, 3, 3), dtype=torch.int32)
    packed, _ = tq_ops.pack_conv_weight(small, "mfma")
    assert tq_ops.mfma_flush_steps(packed, 9) == 0


def test_mfma_flush_chunk_windows_cover_chunk_major_order():
    """kc_chunk (tq_ops.mfma_flush_chunk) bounds every window of consecutive taps of one
    64-channel chunk -- the order the input-patch engine walks -- and a brute-force walk of
    that order with flushes every kc_chunk steps and at chunk ends never exceeds 2^24."""
    import tq_ops  # noqa: F811
    torch.manual_seed(3)
    cin, kh = 256, 3
    codes = torch.randint(-256, 257, (8, cin, kh, kh), dtype=torch.int32)
    codes[:, :64] *= 0  # uneven chunks: the bound must hold per chunk
    packed, cp = tq_ops.pack_conv_weight(codes, "mfma")
    for db in (8, 9):
        kc = tq_ops.mfma_flush_chunk(packed, db, cp, kh * kh)
        assert kc >= 1
        nch = cp // 64
        steps = packed.double().abs().view(packed.shape[0], -1, 64).sum(-1)  # [O, S]
        lim = 2.0**24 / 2**db
        for c in range(nch):
            seq = [steps[:, t * nch + c] for t in range(kh * kh)]
            win = torch.zeros(packed.shape[0], dtype=torch.float64)
            for i, v in enumerate(seq):
                if i % kc == 0:
                    win.zero_()
                win += v
                assert float(win.max()) <= lim
        # one step more would break some window (kc is the largest valid one), unless kc
        # already covers a whole chunk
        if kc < kh * kh:
            assert tq_ops.mfma_flush_chunk(packed, db + 1, cp, kh * kh) <= kc
    assert tq_ops.mfma_flush_chunk(packed[:, :64 * 9], 9, 48, 9) == -1  # Cp % 64 != 0


def test_stem_weight_split_is_exact():
    """pack_stem_weight: two fp16 parts of w * 2^10 summing to the fp32 weight within 2^-22
    relative (2^-35 absolute once the remainder is an fp16 subnormal), in the space-to-depth
    K order of the stem kernel (zero taps where the 8x8 pad is); out-of-range weights are
    refused."""
    import tq_ops  # noqa: F811
    torch.manual_seed(4)
    w = torch.randn(64, 3, 7, 7) * 0.07
    w[0, 0, 0, 0] = 31.9
    w[1, 1, 1, 1] = 3e-7
    parts = tq_ops.pack_stem_weight(w).view(torch.float16).double()  # [2, 64, 192]
    assert tuple(parts.shape) == (2, 64, 192)
    tot = parts.sum(0) * 2.0**-tq_ops.STEM_W_EXP
    w8 = torch.zeros(64, 3, 8, 8, dtype=torch.float64)
    w8[:, :, 1:, 1:] = w.double()
    k = w8.view(64, 3, 4, 2, 4, 2).permute(0, 2, 4, 3, 5, 1).reshape(64, 192)
    bound = 2.0**-22 * k.abs() + 2.0**-35
    assert bool(((tot - k).abs() <= bound).all())
    # K index k = ((sy*4 + sx)*2 + sub_r)*6 + sub_c*3 + c  <->  tap (2sy+sub_r-1, 2sx+sub_c-1)
    for (o, c, r, q) in [(0, 0, 0, 0), (5, 2, 6, 6), (63, 1, 3, 4)]:
        kh8, kw8 = r + 1, q + 1
        idx = ((kh8 // 2 * 4 + kw8 // 2) * 2 + kh8 % 2) * 6 + (kw8 % 2) * 3 + c
        wv = float(w[o, c, r, q])
        assert abs(float(tot[o, idx]) - wv) <= 2.0**-22 * abs(wv) + 2.0**-35
    with pytest.raises(RuntimeError):
        tq_ops.pack_stem_weight(torch.zeros(64, 3, 5, 5))
    for bad in (33.0, float("inf"), float("nan")):
        wb = w.clone()
        wb[3, 2, 1, 0] = bad
        with pytest.raises(RuntimeError, match="finite"):
            tq_ops.pack_stem_weight(wb)


def _hese_masks_np(q):
    hi, lo = q >> 1, q << 1
    a = q & ~hi
    return (a & ~lo) | ((a & lo) << 1), q & hi & ~lo


def _popcount_np(m):
    c = np.zeros_like(m)
    while m.any():
        c += m & 1
        m = m >> 1
    return c


def test_hese_max_terms():
    """csrc/tq_device.h hese_max_terms: the largest HESE term count of a bw-bit magnitude is
    floor(2 (bw + 1) / 3) (the epilogue fast path caps its top-bit peels there)."""
    for bw in range(1, 21):
        pos, neg = _hese_masks_np(np.arange(1 << bw, dtype=np.int64))
        assert _popcount_np(pos | neg).max() == 2 * (bw + 1) // 3, bw


def test_relu_fast_path_restatement():
    """csrc/tq_device.h tr_values_relu4, restated in numpy: the division-free quotient
    fp32(double(y) * RN64(1/sf)), the fract-based rounding and the top-bit peel (capped at
    hese_max_terms) give the oracle's TR value for y >= 0 -- including values placed on and a
    few ulps around every rounding midpoint."""
    rng = np.random.default_rng(0)
    for bw, k in [(9, 3), (9, 0), (9, 1), (9, 12), (8, 8), (11, 4), (4, 2), (14, 5)]:
        maxv = np.float32(2 ** bw - 1)
        for sf in (np.float32(0.037), np.float32(1.0), np.float32(3.3e-5)):
            mids = ((np.arange(0, 2 ** bw + 8) + 0.5) * np.float64(sf)).astype(np.float32)
            around = np.concatenate([mids] + [np.nextafter(mids, np.float32(np.inf) * d)
                                              for d in (1, -1)] +
                                    [np.nextafter(np.nextafter(mids, np.float32(np.inf)),
                                                  np.float32(np.inf))])
            y = np.concatenate([rng.exponential(2.0 ** bw * float(sf) * 0.02, 20000), around,
                                [0.0, np.inf, 1e30]]).astype(np.float32)
            inv = 1.0 / np.float64(sf)
            with np.errstate(over="ignore"):
                t = (y.astype(np.float64) * inv).astype(np.float32)  # quotient_f32
            r = np.minimum(t, maxv)
            fl = np.floor(r)
            q = (fl.astype(np.int64) + ((r - fl) >= 0.5)).astype(np.int64)
            pos, neg = _hese_masks_np(q)
            m = pos | neg
            rest = m.copy()
            for _ in range(min(k, 2 * (bw + 1) // 3)):
                nz = rest > 0
                top = np.zeros_like(rest)
                top[nz] = 1 << np.floor(np.log2(rest[nz])).astype(np.int64)
                rest = rest & ~top
            keep = m ^ rest
            got = (pos & keep) - (neg & keep)
            exp = oracle.tr(y.reshape(1, -1, 1, 1), float(sf), bw, 1, k).reshape(-1) / sf
            np.testing.assert_array_equal(got.astype(np.float64),
                                          np.round(exp.astype(np.float64)))


def test_mfma_flush_nonneg_windows():
    """tq_ops.mfma_flush_steps(nonneg=True) against its spec by brute force: the largest n
    with max(sum of positive v_w, sum of |negative v_w|) * 2^db <= 2^24 over every window of
    n K-steps of every row; never narrower than the general (sum |v_w|) window."""
    import tq_ops  # noqa: F811
    g = torch.Generator().manual_seed(3)
    for trial in range(6):
        o, steps = 5, 12
        v = torch.randint(-256, 257, (o, steps * 64), generator=g).double()
        if trial % 2:
            v[:, : steps * 32] = v[:, : steps * 32].abs()  # sign-skewed rows
        db = 9
        lim = 2.0**24 / 2**db
        st = v.view(o, steps, 64)
        pos, neg = st.clamp(min=0).sum(-1), (-st).clamp(min=0).sum(-1)

        def ok(n):
            return all(max(float(pos[r, i:i + n].sum()), float(neg[r, i:i + n].sum())) <= lim
                       for r in range(o) for i in range(steps - n + 1))
        best = max([n for n in range(1, steps + 1) if ok(n)], default=0)
        exp = -1 if best == 0 else (0 if best == steps else best)
        got = tq_ops.mfma_flush_steps(v, db, nonneg=True)
        assert got == exp, (trial, got, exp)
        gen = tq_ops.mfma_flush_steps(v, db)
        assert gen != -1 or got == -1
        if gen > 0:
            assert got == 0 or got >= gen


def test_mfma_flush_chunk_nonneg_brute_force():
    """mfma_flush_chunk(nonneg=True) against its spec by brute force, in the chunk-major
    order the input-patch engine walks (each 64-channel chunk, all taps)."""
    import tq_ops  # noqa: F811
    g = torch.Generator().manual_seed(9)
    for trial in range(5):
        cout, cin, kh = 6, 192, 3
        codes = torch.randint(-256, 257, (cout, cin, kh, kh), generator=g, dtype=torch.int32)
        if trial % 2:
            codes[:, :96] = codes[:, :96].abs()
        packed, cp = tq_ops.pack_conv_weight(codes, "mfma")
        db = 9
        lim = 2.0**24 / 2**db
        nch, ntaps = cp // 64, kh * kh
        st = packed.double().view(packed.shape[0], -1, 64)  # [O, tap * nch + c, 64]
        pos, neg = st.clamp(min=0).sum(-1), (-st).clamp(min=0).sum(-1)

        def ok(n):
            for c in range(nch):
                for i in range(ntaps - n + 1):
                    taps = [(i + t) * nch + c for t in range(n)]
                    if max(float(pos[:, taps].sum(1).max()), float(neg[:, taps].sum(1).max())) \
                            > lim:
                        return False
            return True
        best = max([n for n in range(1, ntaps + 1) if ok(n)], default=0)
        exp = -1 if best == 0 else (0 if best == ntaps else best)
        assert tq_ops.mfma_flush_chunk(packed, db, cp, ntaps, nonneg=True) == exp
        gen = tq_ops.mfma_flush_chunk(packed, db, cp, ntaps)
        if gen > 0:
            assert exp == 0 or exp >= gen
