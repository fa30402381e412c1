"""GPU parity of the tracking-histogram kernel (tq_histc_f32, tr_layer.py:91-94).

Counts are integers, so the bar is bit-exact: against the oracle's restatement of
torch.histc (oracle.histc) on every input, and against torch.histc itself on the GPU wherever
its fp32 atomic counts are still exact (every bin < 2^24)."""
import numpy as np
import pytest
import torch

import oracle
import tq_ops
import tr_layer

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _track(x, nbins, minv, maxv, hist=None):
    hist = torch.zeros(nbins, dtype=torch.float32, device=DEV) if hist is None else hist
    counts = torch.zeros(nbins, dtype=torch.int64, device=DEV)
    tq_ops.histc_track(x, hist, minv, maxv, counts)
    assert int(counts.abs().sum()) == 0  # the scratch is left zeroed
    return hist


def _edges_input(nbins, minv, maxv, n_random, seed):
    rng = np.random.default_rng(seed)
    lo, hi = np.float32(minv), np.float32(maxv)
    edges = lo + np.arange(nbins + 1, dtype=np.float32) * ((hi - lo) / np.float32(nbins))
    return np.concatenate([
        rng.standard_normal(n_random).astype(np.float32) * (hi - lo) / 3 + (hi + lo) / 2,
        edges, np.nextafter(edges, np.float32(-np.inf)), np.nextafter(edges, np.float32(np.inf)),
        np.array([lo, hi, np.inf, -np.inf, np.nan, 1e30, -1e30, 0.0, -0.0], np.float32)])


@pytest.mark.parametrize("nbins,minv,maxv", [(8192, -50, 50), (1000, -3, 7), (37, 0, 1),
                                             (20000, -50, 50)])
@pytest.mark.parametrize("tail", [0, 1, 3])
def test_histc_bit_exact(nbins, minv, maxv, tail):
    x = _edges_input(nbins, minv, maxv, (1 << 18) + tail, nbins)
    xt = torch.from_numpy(x).to(DEV)
    got = _track(xt, nbins, minv, maxv).cpu().numpy().astype(np.int64)
    np.testing.assert_array_equal(got, oracle.histc(x, nbins, minv, maxv))
    ref = torch.histc(xt, nbins, minv, maxv).cpu().numpy().astype(np.int64)
    np.testing.assert_array_equal(got, ref)


def test_histc_relu_activation_layouts_and_accumulation():
    """A post-ReLU NCHW activation and its channels_last copy (same multiset of values) give
    the same histogram; a second call adds to the first (hist_bins +=)."""
    torch.manual_seed(0)
    x = torch.relu(torch.randn(16, 64, 28, 28, device=DEV) * 2)
    h1 = _track(x, 8192, -50, 50)
    h2 = _track(x.contiguous(memory_format=torch.channels_last), 8192, -50, 50)
    assert torch.equal(h1, h2)
    np.testing.assert_array_equal(h1.cpu().numpy().astype(np.int64),
                                  oracle.histc(x.cpu().numpy(), 8192, -50, 50))
    _track(x, 8192, -50, 50, hist=h1)
    assert torch.equal(h1, 2 * h2)
    # strided (non-dense) and misaligned views go through a dense copy
    xs = x[:, ::2]
    np.testing.assert_array_equal(_track(xs, 8192, -50, 50).cpu().numpy().astype(np.int64),
                                  oracle.histc(xs.cpu().numpy(), 8192, -50, 50))
    xo = x.view(-1)[1:4097]
    np.testing.assert_array_equal(_track(xo, 8192, -50, 50).cpu().numpy().astype(np.int64),
                                  oracle.histc(xo.cpu().numpy(), 8192, -50, 50))


def test_histc_counts_past_fp32_exact_range():
    """The zero bin of a 256-image layer-1 ReLU output holds ~25 M elements, past 2^24: the
    kernel's count is exact (torch.histc's fp32 atomic counts are not)."""
    n = (1 << 24) + 12345
    x = torch.zeros(n + 1000, device=DEV)
    x[n:] = 1.0
    h = _track(x, 8192, -50, 50)
    b0 = oracle.histc(np.zeros(1, np.float32), 8192, -50, 50).argmax()
    b1 = oracle.histc(np.ones(1, np.float32), 8192, -50, 50).argmax()
    assert h[b0].item() == float(np.float32(n))
    assert h[b1].item() == 1000.0
    assert h.sum().item() == float(np.float32(n)) + 1000.0


def test_linear_quantize_tracking_uses_kernel():
    """LinearQuantize in tracking mode: the histogram equals torch.histc's (small counts) and
    the calibrated sf equals the one computed from torch.histc's histogram."""
    torch.manual_seed(1)
    q = tr_layer.LinearQuantize(9, 3).to(DEV)
    ref = torch.zeros(8192, device=DEV)
    for _ in range(3):
        x = torch.relu(torch.randn(8, 32, 14, 14, device=DEV))
        assert q(x) is x
        ref += torch.histc(x, 8192, -50, 50)
    assert torch.equal(q.hist_bins, ref)
    sf_ref = tr_layer.mse_profile(ref, -50, 50, 9, 3)
    q.finish_tracking()
    assert q.sf == sf_ref
