"""GPU parity of the TR op (libtq_hip.so through the reference API) against the oracle.

Bit-exact (torch.equal) on every case: the encode/select/rescale path is integer work plus
one fp32 (fp64) multiply, so any difference is a bug."""
import numpy as np
import pytest
import torch

import oracle
import tq_native
import tq_ops
import tr_layer

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _gpu_tr(x, sf, bw, g, k):
    return tr_layer.tr_cuda.tr(torch.from_numpy(x).to(DEV), sf, bw, g, k).cpu().numpy()


def assert_bit_equal(got, exp):
    """Bitwise equality; NaNs only need to be NaN (0 * inf payloads differ across ISAs)."""
    nan = np.isnan(exp)
    assert np.array_equal(np.isnan(got), nan)
    np.testing.assert_array_equal(got[~nan].view(np.uint8), exp[~nan].view(np.uint8))


def _check(x, sf, bw, g, k):
    got = _gpu_tr(x, sf, bw, g, k)
    exp = oracle.tr(x, sf, bw, g, k)
    assert_bit_equal(got, exp)


SHAPES = [(8, 16, 3, 3), (16, 32, 1, 1), (10, 32), (1, 4096, 1, 1), (3, 10), (5, 37, 2, 3),
          (2, 64, 7, 5)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("g,k", [(1, 0), (1, 1), (1, 3), (2, 3), (8, 12), (16, 24), (32, 96),
                                 (8, 1), (3, 5)])
def test_tr_matches_oracle_f32(shape, g, k):
    rng = np.random.default_rng(hash((shape, g, k)) % 2**32)
    x = (rng.standard_normal(shape) * 1.5).astype(np.float32)
    sf = float(np.abs(x).max()) / 2**8  # the weight scale rule, tr_layer.py:118-119
    _check(x, sf, 9, g, k)


@pytest.mark.parametrize("bw", [0, 1, 4, 8, 9, 16, 24])
def test_tr_bitwidths(bw):
    rng = np.random.default_rng(bw)
    x = (rng.standard_normal((4, 48, 3, 3)) * 4).astype(np.float32)
    for g, k in [(1, 3), (8, 12), (32, 96)]:
        _check(x, float(np.abs(x).max()) / 2 ** max(bw - 1, 0), bw, g, k)


def test_tr_edge_values():
    base = np.array([np.float32(0.49999997), 0.5, 1.5, 2.5, -0.5, -0.0, 0.0, 1e30, -1e30,
                     np.inf, -np.inf, np.nan, 511.49, 511.5, 1e-40, -3.0000002], np.float32)
    x = np.tile(base, 4).reshape(4, 16)
    for sf in [1.0, 1e-8, 0.0, np.inf, 0.37]:
        for g, k in [(1, 9), (1, 2), (8, 12), (16, 3)]:
            _check(x, sf, 9, g, k)


def test_tr_f64_matches_oracle():
    rng = np.random.default_rng(11)
    x = rng.standard_normal((6, 24, 3, 3)) * 3
    for g, k in [(1, 3), (8, 12), (32, 96)]:
        _check(x, float(np.abs(x).max()) / 256, 9, g, k)


@pytest.mark.parametrize("shape", [(2, 3, 4), (2, 3, 4, 5, 2), (4, 7)])
def test_tr_shape_rules(shape):
    rng = np.random.default_rng(5)
    x = rng.standard_normal(shape).astype(np.float32)
    _check(x, 0.05, 8, 1, 3)
    _check(x, 0.05, 8, 2, 3)


def test_tr_activation_full_size_bit_exact():
    """D1 workload: relu(N(0,1)) 256x64x56x56, sf=0.05, db=9, dt=3, g=1,
    viewed (1,-1,1,1) -- bit-exact against the oracle over all 51,380,224 elements."""
    torch.manual_seed(0)
    x = torch.relu(torch.randn(256, 64, 56, 56, device=DEV))
    got = tr_layer.tr_cuda.tr(x.view(1, -1, 1, 1), 0.05, 9, 1, 3)
    exp = oracle.tr(x.view(1, -1, 1, 1).cpu().numpy(), 0.05, 9, 1, 3)
    assert torch.equal(got.cpu(), torch.from_numpy(exp))


def test_tr_encode_codes_consistent():
    rng = np.random.default_rng(2)
    w = torch.from_numpy((rng.standard_normal((32, 64, 3, 3)) * 0.1).astype(np.float32))
    sf = w.abs().max().item() / 256
    out, codes = tq_ops.tr_encode(w.to(DEV), sf, 9, 8, 12)
    exp = oracle.tr(w.numpy(), sf, 9, 8, 12)
    assert torch.equal(out.cpu(), torch.from_numpy(exp))
    assert torch.equal(codes.cpu().float() * np.float32(sf), out.cpu())


def test_tr_errors_mirror_reference():
    # (CPU tensors are the host library's: tests/test_host_tr.py)
    with pytest.raises(RuntimeError, match="CUDA"):
        tr_layer.tr_cuda.tr(torch.zeros(2, 2, device="meta"), 1.0, 8, 1, 1)
    with pytest.raises(RuntimeError, match="contiguous"):
        tr_layer.tr_cuda.tr(torch.zeros(4, 4, device=DEV).t(), 1.0, 8, 1, 1)
    with pytest.raises(RuntimeError):
        tr_layer.tr_cuda.tr(torch.zeros(2, 2, dtype=torch.int32, device=DEV), 1.0, 8, 1, 1)
    with pytest.raises(IndexError):
        tr_layer.tr_cuda.tr(torch.zeros(4, device=DEV), 1.0, 8, 1, 1)
    with pytest.raises(RuntimeError, match="group_size"):
        tr_layer.tr_cuda.tr(torch.zeros(2, 64, device=DEV), 1.0, 8, 33, 1)
    assert tr_layer.tr_cuda.tr(torch.zeros(0, 4, device=DEV), 1.0, 8, 1, 1).shape == (0, 4)


def test_tr_elementwise_channels_last():
    torch.manual_seed(3)
    x = torch.randn(4, 24, 5, 7, device=DEV).to(memory_format=torch.channels_last)
    got = tq_ops.tr_elementwise(x, 0.03, 9, 3)
    assert got.is_contiguous(memory_format=torch.channels_last)
    exp = oracle.tr(x.contiguous().view(1, -1, 1, 1).cpu().numpy(), 0.03, 9, 1, 3)
    assert torch.equal(got.contiguous().view(1, -1, 1, 1).cpu(), torch.from_numpy(exp))


def test_tr_on_side_stream_orders_with_torch():
    s = torch.cuda.Stream()
    x = torch.randn(64, 512, device=DEV)
    with torch.cuda.stream(s):
        y = tr_layer.tr_cuda.tr(x * 2, 0.01, 9, 8, 12)
        z = y + 0
    torch.cuda.synchronize()
    exp = oracle.tr((x * 2).cpu().numpy(), 0.01, 9, 8, 12)
    assert torch.equal(z.cpu(), torch.from_numpy(exp))


def test_mse_profile_device_equals_host():
    """The calibration kernel and the host library sum the same fp32 per-bin errors in the
    same fp64 order (no fma contraction on either side): identical errs, identical sf."""
    import tq_native
    torch.manual_seed(5)
    hist = torch.histc(torch.relu(torch.randn(300000)) * 5, 8192, -50, 50)
    x = torch.linspace(-50, 50, 8192)
    sfs = torch.tensor(torch.linspace(1e-8, 50, 2048).tolist(), dtype=torch.float32)
    for bits, terms in [(9, 3), (8, 8), (4, 2)]:
        dev = tq_native.mse_profile(x.to(DEV), hist.to(DEV), sfs.to(DEV), bits, terms)
        host = tq_native.mse_profile_host(x, hist, sfs, bits, terms)
        assert torch.equal(dev.cpu(), host)
        assert tr_layer.mse_profile(hist.to(DEV), -50, 50, bits, terms) == \
            tr_layer.mse_profile(hist, -50, 50, bits, terms)


def test_mse_profile_matches_oracle():
    torch.manual_seed(4)
    hist = torch.histc(torch.relu(torch.randn(200000)) * 3, 8192, -50, 50)
    for bits, terms in [(9, 3), (8, 8), (6, 6)]:
        sf = tr_layer.mse_profile(hist.to(DEV), -50, 50, bits, terms)
        sf_ref, errs = oracle.mse_profile(hist.numpy(), -50, 50, bits, terms)
        if sf != sf_ref:
            # only a tie in the error (fp64 restatement vs kernel order) may move the argmin
            idx = torch.linspace(1e-8, 50, 2048).tolist().index(sf)
            assert abs(errs[idx] - errs.min()) <= 1e-9 * max(errs.min(), 1e-30)


def test_library_version():
    assert tq_native.version().startswith("tq-hip")


def _near_midpoints(rng, qmax, n_sf=64, per_sf=512):
    """fp32 inputs whose quotient |x|/sf lies within a few ulps of a rounding midpoint
    q + 0.5 of the quantizer, for random fp32 scales (normal, tiny and huge) -- the cases
    where a wrong fp32 quotient would change q."""
    sfs = np.concatenate([rng.uniform(1e-3, 1.0, n_sf // 2),
                          10.0 ** rng.uniform(-30, 30, n_sf // 2)]).astype(np.float32)
    out = []
    for sf in sfs:
        q = rng.integers(0, qmax, per_sf).astype(np.float64)
        mid = ((q + 0.5) * np.float64(sf)).astype(np.float32)
        steps = rng.integers(-3, 4, per_sf).astype(np.int32)
        x = mid.view(np.int32) + steps
        x = x.view(np.float32)
        x = np.where(rng.random(per_sf) < 0.5, -x, x).astype(np.float32)
        out.append((float(sf), x))
    return out


@pytest.mark.parametrize("bw", [9, 24])
def test_tr_quotient_near_midpoints(bw):
    """The division-free quantizer (fp32(|x| * RN64(1/sf)), tq_device.h) against the
    oracle's true fp32 division, on quotients a few ulps from every kind of midpoint."""
    rng = np.random.default_rng(bw)
    for sf, x in _near_midpoints(rng, 2**bw):
        x = x.reshape(1, -1, 1, 1)
        for k in (3, 24):
            _check(x, sf, bw, 1, k)
        _check(x.reshape(-1, 8), sf, bw, 8, 12)


def test_act_codes_near_midpoints():
    """Activation codes (tq_act_encode, the epilogue's TR) on the same adversarial inputs."""
    rng = np.random.default_rng(5)
    for sf, x in _near_midpoints(rng, 2**14, n_sf=16, per_sf=64 * 16):
        xt = torch.from_numpy(x.reshape(16, 64, 1, 1)).to(DEV).contiguous(
            memory_format=torch.channels_last)
        codes = torch.empty((16, 1, 1, 64), dtype=torch.int16, device=DEV)
        tq_native.act_encode(xt, True, sf, 14, 3, codes)
        exp = oracle.tr(x.reshape(1, -1, 1, 1), sf, 14, 1, 3).reshape(16, 64)
        got = codes.cpu().numpy().reshape(16, 64).astype(np.float32) * np.float32(sf)
        np.testing.assert_array_equal(got, exp)


def _random_case(rng):
    """One seeded random TR case: shape (rank 2-4; ragged last groups half the time), group
    (<= 32, the reference's limit), kept terms, bit width, scale and a value mix with ties,
    tails and specials."""
    g = int(rng.choice([1, 2, 3, 4, 8, 16, 32]))
    k = int(rng.integers(0, 3 * g + 1))
    bw = int(rng.integers(1, 17))
    c = g * int(rng.integers(1, max(2, 256 // g))) + (int(rng.integers(0, g)) if rng.random() < 0.5 else 0)
    rank = int(rng.integers(2, 5))
    shape = (int(rng.integers(1, 9)), c) + tuple(int(rng.integers(1, 13)) for _ in range(rank - 2))
    kind = int(rng.integers(0, 4))
    n = int(np.prod(shape))
    if kind == 0:
        x = rng.standard_normal(n) * float(10.0 ** rng.uniform(-3, 3))
    elif kind == 1:
        x = rng.laplace(size=n) * float(10.0 ** rng.uniform(-2, 2))
    elif kind == 2:
        x = np.maximum(rng.standard_normal(n), 0.0)  # post-ReLU activations
    else:
        x = (rng.integers(-2 ** bw, 2 ** bw, n) + rng.choice([0.0, 0.5], n)).astype(np.float64)
    qmax = float(2 ** bw - 1) if bw else 1.0
    if kind == 3:
        sf = float(rng.choice([1.0, 0.5, 0.25]))  # exact midpoints of the quantizer
    else:
        sf = float(np.abs(x).max()) / qmax * float(rng.choice([1.0, 0.5, 2.0])) or 1.0
    special = rng.random(n) < 0.01
    x[special] = rng.choice([0.0, -0.0, np.inf, -np.inf, np.nan, 1e30], int(special.sum()))
    dtype = np.float64 if rng.random() < 0.25 else np.float32
    return x.reshape(shape).astype(dtype), sf, bw, g, k


@pytest.mark.parametrize("seed", range(48))
def test_tr_random_sweep(seed):
    """Seeded random sweep over shapes, groups, kept terms, bit widths 1-16, fp32 / fp64,
    scales (incl. exact quantizer midpoints) and special values: bit-exact against the
    oracle (the reference's tr kernel, kernels/tr_cuda_kernel.cu, restated in oracle/)."""
    x, sf, bw, g, k = _random_case(np.random.default_rng(1000 + seed))
    _check(x, sf, bw, g, k)
