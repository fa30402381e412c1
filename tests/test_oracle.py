"""Pin the CPU oracle against the reference's own outputs (CPU-only).

The oracle (oracle/tr_oracle.c) is the checker for every GPU parity test, so it is pinned
first: its HESE encoder against golden vectors produced by the reference's bit_utils.hese
(tests/golden/gen_golden.py), and its selection against an independent sorted-top-k
restatement of the reference greedy."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _closed_form(q):
    """The device formula of term-quantization_amd/csrc/tq_device.h hese_masks, in numpy."""
    q = np.asarray(q, dtype=np.uint64)
    hi, lo = q >> np.uint64(1), (q << np.uint64(1)) & np.uint64(0xFFFFFFFF)
    a = q & ~hi
    pos = (a & ~lo) | ((a & lo) << np.uint64(1))
    neg = q & hi & ~lo
    return pos.astype(np.uint32), neg.astype(np.uint32)


def test_oracle_hese_matches_bit_utils_golden():
    g = np.load(os.path.join(GOLDEN, "hese_bit_utils.npz"))
    pos, neg = oracle.hese_masks(np.abs(g["q"]))
    neg_q = g["q"] < 0
    # bit_utils.hese(-q) == -bit_utils.hese(q): swap the masks for negative q
    exp_pos = np.where(neg_q, g["neg"], g["pos"])
    exp_neg = np.where(neg_q, g["pos"], g["neg"])
    np.testing.assert_array_equal(pos, exp_pos)
    np.testing.assert_array_equal(neg, exp_neg)


def test_oracle_term_order_matches_bit_utils():
    # a few full term lists (order and sign), the form bit_utils.hese returns
    assert oracle.hese_terms(0) == []
    assert oracle.hese_terms(3) == [4, -1]
    assert oracle.hese_terms(11) == [8, 4, -1]
    assert oracle.hese_terms(511) == [512, -1]
    assert oracle.hese_terms(-5) == [-4, -1]


def test_python_hese_restatement_matches_golden_and_c():
    """oracle.hese_py (BASELINE C1's Python baseline) = the golden bit_utils.hese masks and
    the C encoder's term lists (order and sign)."""
    g = np.load(os.path.join(GOLDEN, "hese_bit_utils.npz"))
    for q, p, n in zip(g["q"].tolist(), g["pos"].tolist(), g["neg"].tolist()):
        terms = oracle.hese_py(q)
        sp = sum(1 << (abs(t).bit_length() - 1) for t in terms if t > 0)
        sn = sum(1 << (abs(t).bit_length() - 1) for t in terms if t < 0)
        assert (sp, sn) == (p, n), q
    rng = np.random.default_rng(3)
    for q in list(range(-1100, 1100)) + rng.integers(-(1 << 22), 1 << 22, 500).tolist():
        assert oracle.hese_py(q) == oracle.hese_terms(q), q


@pytest.mark.parametrize("g,k", [(8, 12), (1, 3), (4, 5), (16, 20), (8, 0)])
def test_python_tr_restatement_matches_c(g, k):
    """oracle.tr_py (BASELINE C2's Python baseline) is bit-identical to the C restatement on a
    flat (1, C) tensor, partial last group and clamped values included."""
    rng = np.random.default_rng(g * 100 + k)
    x = (rng.standard_normal(3000) * 3).astype(np.float32)
    x[::97] = 0.0
    x[5] = 1e9  # clamps to 2^b - 1
    a = oracle.tr_py(x, 0.05, 9, g, k)
    b = oracle.tr(x.reshape(1, -1), 0.05, 9, g, k).reshape(-1)
    np.testing.assert_array_equal(a.view(np.int32), b.view(np.int32))


def test_closed_form_hese_full_table_sha256():
    """Every q < 2^17 through the device closed form hashes to the bit_utils.hese table."""
    meta = json.load(open(os.path.join(GOLDEN, "hese_bit_utils_sha256.json")))
    lo, hi = meta["q_range"]
    pos, neg = _closed_form(np.arange(lo, hi))
    digest = hashlib.sha256(pos.astype("<u4").tobytes() + neg.astype("<u4").tobytes())
    assert digest.hexdigest() == meta["sha256"]


def test_closed_form_matches_oracle_encoder():
    qs = np.arange(0, 4096)
    p1, n1 = oracle.hese_masks(qs)
    p2, n2 = _closed_form(qs)
    np.testing.assert_array_equal(p1, p2)
    np.testing.assert_array_equal(n1, n2)


def _sorted_topk_tr(x, sf, bw, g, k):
    """Independent restatement of the reference selection (kernels/tr_cuda_kernel.cu:92-116)
    as a sort: keep the first k terms of a group by (exponent desc, channel asc)."""
    x = np.asarray(x, np.float32)
    B, C = x.shape
    out = np.zeros_like(x)
    maxv = np.float32(2.0 ** bw - 1)
    sf32 = np.float32(sf)
    for b in range(B):
        for c0 in range(0, C, g):
            terms = []
            for j in range(c0, min(c0 + g, C)):
                t = float(np.float32(abs(x[b, j]) / sf32)) + 0.5
                q = int(min(t, float(maxv))) if t == t else 0
                sign = -1 if x[b, j] < 0 else 1
                for tv in oracle.hese_terms(q):
                    terms.append((-abs(tv), j, sign * tv))
            terms.sort()
            acc = {}
            for _, j, tv in terms[:max(k, 0)]:
                acc[j] = acc.get(j, 0) + tv
            for j in range(c0, min(c0 + g, C)):
                out[b, j] = np.float32(acc.get(j, 0)) * sf32
    return out


@pytest.mark.parametrize("g,k", [(1, 1), (1, 3), (2, 3), (8, 12), (8, 0), (16, 24), (32, 96)])
def test_oracle_greedy_equals_sorted_topk(g, k):
    rng = np.random.default_rng(1234 + g * 100 + k)
    x = (rng.standard_normal((6, 64)) * 2).astype(np.float32)
    sf = 4.0 / 256
    got = oracle.tr(x, sf, 9, g, k)
    np.testing.assert_array_equal(got, _sorted_topk_tr(x, sf, 9, g, k))


def test_oracle_rounding_traps():
    sf = np.float32(1.0)
    # 0.49999997f rounds to 0 with the reference's double +0.5 (1 with an fp32 +0.5f)
    x = np.array([[np.float32(0.49999997), 0.5, 1.5, 2.5, -0.5, -0.0, 0.0]], np.float32)
    got = oracle.tr(x, sf, 9, 1, 9)
    np.testing.assert_array_equal(got, np.array([[0, 1, 2, 3, -1, 0, 0]], np.float32))
    # saturation and NaN: huge / inf clamp to 2^bw - 1, NaN -> 0
    x = np.array([[1e30, np.inf, -np.inf, np.nan]], np.float32)
    got = oracle.tr(x, np.float32(1e-8), 4, 1, 9)
    v = np.float32(15) * np.float32(1e-8)
    np.testing.assert_array_equal(got, np.array([[v, v, -v, 0]], np.float32))


def test_oracle_partial_last_group():
    # C % g != 0: the last group is [8, 10) -- defined here, racy in the reference
    rng = np.random.default_rng(7)
    x = rng.standard_normal((3, 10)).astype(np.float32)
    got = oracle.tr(x, 0.02, 9, 8, 4)
    np.testing.assert_array_equal(got, _sorted_topk_tr(x, 0.02, 9, 8, 4))


def test_oracle_shape_rules():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((2, 3, 4)).astype(np.float32)  # 3-D: only first B*C processed
    got = oracle.tr(x, 0.05, 8, 1, 3)
    flat = x.reshape(-1)
    exp = np.zeros_like(flat)
    exp[:6] = oracle.tr(flat[:6].reshape(2, 3), 0.05, 8, 1, 3).reshape(-1)
    np.testing.assert_array_equal(got.reshape(-1), exp)


def test_oracle_ubsan_clean(tmp_path):
    """The restatement has no undefined shifts/overflows (host UBSan build)."""
    import ctypes
    import subprocess
    here = os.path.dirname(oracle.__file__)
    r = subprocess.run(["make", "-s", "-C", here, "liboracle_ubsan.so"], capture_output=True)
    if r.returncode != 0:
        pytest.skip("UBSan runtime unavailable: %s" % r.stderr.decode()[-200:])
    code = (
        "import ctypes, numpy as np, sys\n"
        "l = ctypes.CDLL(%r)\n"
        "x = (np.random.default_rng(0).standard_normal((4, 64)) * 40).astype(np.float32)\n"
        "o = np.empty_like(x); s = (ctypes.c_int64 * 2)(4, 64)\n"
        "fp = ctypes.POINTER(ctypes.c_float)\n"
        "for bw, g, k in [(16, 8, 12), (24, 32, 96), (9, 1, 3)]:\n"
        "    rc = l.oracle_tr_f32(x.ctypes.data_as(fp), o.ctypes.data_as(fp), 2, s,"
        " ctypes.c_float(1e-3), bw, g, k)\n"
        "    assert rc == 0\n" % os.path.join(here, "liboracle_ubsan.so"))
    r = subprocess.run(["python", "-c", code], capture_output=True)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    assert b"runtime error" not in r.stderr


@pytest.mark.parametrize("nbins,minv,maxv", [(8192, -50, 50), (1000, -3, 7), (37, 0, 1)])
def test_oracle_histc_matches_torch_histc(nbins, minv, maxv):
    """The histogram restatement behind the tracking-kernel tests equals torch.histc (the
    reference's call, tr_layer.py:91-94) on random values, every bin edge and its fp32
    neighbours, the range ends, out-of-range values, infinities and NaN."""
    import torch
    rng = np.random.default_rng(nbins)
    lo, hi = np.float32(minv), np.float32(maxv)
    edges = (lo + np.arange(nbins + 1, dtype=np.float32) * ((hi - lo) / np.float32(nbins)))
    x = np.concatenate([
        rng.standard_normal(1 << 16).astype(np.float32) * (hi - lo) / 2 + (hi + lo) / 2,
        edges, np.nextafter(edges, np.float32(-np.inf)), np.nextafter(edges, np.float32(np.inf)),
        np.array([lo, hi, np.inf, -np.inf, np.nan, 1e30, -1e30], np.float32)]).astype(np.float32)
    got = oracle.histc(x, nbins, minv, maxv)
    exp = torch.histc(torch.from_numpy(x), nbins, minv, maxv).numpy().astype(np.int64)
    np.testing.assert_array_equal(got, exp)
