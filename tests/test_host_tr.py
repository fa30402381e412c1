"""The product CPU path: libtq_host.so (include/tq_host.h) -- CPU-only, no GPU needed.

The reference's MNIST config runs on CPU torch (evaluate_mlp.py:56-57) but its TR extension
rejects CPU tensors (kernels/tr_cuda.cpp:12-18).  The host library is the product TR op for
CPU tensors; it is a different design from the oracle (closed-form HESE +
threshold selection, OpenMP), so every result is checked bit-exact against the oracle over
the SURVEY 8(c) fixture matrix, and its calibration errors against a numpy restatement with
the same summation order."""
import ctypes
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.nn as nn

import oracle
import tq_native
import tq_ops
import tr_layer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"\b(tq_[a-z0-9_]+)\s*\(", src)))


def test_host_library_exports_every_declared_symbol():
    lib = tq_native.host_lib()
    declared = _declared("tq_host.h")
    assert declared
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(tq_native.HOST_EXPORTED_SYMBOLS) == declared
    assert lib.tq_host_version().startswith(b"tq-host")


def _host_tr(x, sf, bw, g, k, threads=0):
    t = torch.from_numpy(np.ascontiguousarray(x))
    out = torch.empty_like(t)
    shape = (ctypes.c_int64 * t.dim())(*t.shape)
    fn = tq_native.host_lib().tq_tr_f32_host if t.dtype == torch.float32 else \
        tq_native.host_lib().tq_tr_f64_host
    rc = fn(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(out.data_ptr()), t.dim(), shape,
            float(np.float32(sf)), bw, g, k, threads)
    assert rc == 0, tq_native.host_lib().tq_host_last_error()
    return out.numpy()


SHAPES = [(8, 16, 3, 3), (16, 32, 1, 1), (10, 32), (1, 4096, 1, 1), (3, 10), (2, 650),
          (4, 37, 2, 3)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("g,k", [(1, 0), (1, 1), (1, 3), (2, 3), (3, 5), (8, 12), (8, 1),
                                 (16, 24), (32, 96), (32, 3)])
@pytest.mark.parametrize("bw", [4, 8, 9, 16])
def test_host_tr_bit_exact_vs_oracle(shape, g, k, bw):
    rng = np.random.default_rng(hash((shape, g, k, bw)) % 2**32)
    x = (rng.standard_normal(shape) * rng.choice([0.05, 1.0, 30.0])).astype(np.float32)
    sf = float(np.abs(x).max()) / 2 ** (bw - 1)
    np.testing.assert_array_equal(_host_tr(x, sf, bw, g, k), oracle.tr(x, sf, bw, g, k))


@pytest.mark.parametrize("g,k", [(1, 3), (8, 12), (5, 7)])
def test_host_tr_f64_bit_exact(g, k):
    rng = np.random.default_rng(11)
    x = rng.standard_normal((6, 40, 3, 3)) * 3
    np.testing.assert_array_equal(_host_tr(x, 0.013, 9, g, k), oracle.tr(x, 0.013, 9, g, k))


def test_host_tr_edge_values():
    sf = np.float32(1.0)
    x = np.array([[np.float32(0.49999997), 0.5, 1.5, 2.5, -0.5, -0.0, 0.0, 1e30, np.inf,
                   -np.inf, np.nan, 511.49997, 511.5, 1e-45]], np.float32)
    for bw, g, k in [(9, 1, 9), (4, 1, 9), (9, 2, 3), (16, 7, 5), (0, 1, 3), (24, 1, 24)]:
        for s in (sf, np.float32(1e-8), np.float32(0.0), np.float32(np.inf), np.float32(3e38)):
            np.testing.assert_array_equal(_host_tr(x, s, bw, g, k), oracle.tr(x, s, bw, g, k))
    # near every rounding midpoint of the quotient: +-3 ulps around q + 0.5
    q = np.arange(0, 600, dtype=np.float32) + np.float32(0.5)
    near = np.concatenate([np.nextafter(q, np.float32(np.inf) * s) for s in (1, -1)] + [q])
    for sfv in (np.float32(1.0), np.float32(0.37), np.float32(3.1e-3)):
        x = (near * sfv).astype(np.float32).reshape(1, -1)
        np.testing.assert_array_equal(_host_tr(x, sfv, 10, 1, 4), oracle.tr(x, sfv, 10, 1, 4))


def test_host_tr_shape_rules_and_threads():
    rng = np.random.default_rng(3)
    for shape in [(2, 3, 4), (2, 3, 4, 5, 2), (5, 1), (1, 1, 1, 1)]:
        x = rng.standard_normal(shape).astype(np.float32)
        np.testing.assert_array_equal(_host_tr(x, 0.05, 8, 2, 3), oracle.tr(x, 0.05, 8, 2, 3))
    x = rng.standard_normal((64, 96, 5, 5)).astype(np.float32)
    ref = _host_tr(x, 0.01, 9, 8, 12, threads=1)
    for t in (2, 3, 8):
        np.testing.assert_array_equal(_host_tr(x, 0.01, 9, 8, 12, threads=t), ref)


@pytest.mark.parametrize("args,code,msg", [
    (dict(bw=25), 2, b"bitwidth"), (dict(bw=-1), 2, b"bitwidth"), (dict(g=0), 1, b"group_size"),
    (dict(g=33), 1, b"group_size"), (dict(sf=-1.0), 1, b"sf"), (dict(sf=float("nan")), 1, b"sf"),
])
def test_host_argument_validation(args, code, msg):
    lib = tq_native.host_lib()
    shape = (ctypes.c_int64 * 2)(4, 8)
    p = dict(bw=8, g=1, sf=1.0)
    p.update(args)
    assert lib.tq_tr_f32_host(None, None, 2, shape, p["sf"], p["bw"], p["g"], 1, 0) == code
    assert msg in lib.tq_host_last_error()
    assert lib.tq_tr_f32_host(None, None, 1, shape, 1.0, 8, 1, 1, 0) == 1
    assert b"2 dimensions" in lib.tq_host_last_error()


def test_tq_ops_dispatches_cpu_tensors_to_the_host_library():
    torch.manual_seed(0)
    w = torch.randn(16, 32, 3, 3) * 0.05
    sf = w.abs().max().item() / 256
    got = tr_layer.tr_cuda.tr(w, sf, 9, 8, 12)
    assert got.device.type == "cpu" and got.dtype == torch.float32
    assert torch.equal(got, torch.from_numpy(oracle.tr(w.numpy(), sf, 9, 8, 12)))
    out, codes = tq_ops.tr_encode(w, sf, 9, 8, 12)
    assert torch.equal(out, got)
    assert torch.equal(codes.float() * torch.tensor(np.float32(sf)), got)
    x = torch.relu(torch.randn(2, 8, 5, 5)).to(memory_format=torch.channels_last)
    y = tq_ops.tr_elementwise(x, 0.05, 9, 3)
    exp = oracle.tr(x.contiguous().numpy().reshape(1, -1, 1, 1), 0.05, 9, 1, 3)
    assert torch.equal(y.contiguous(), torch.from_numpy(exp).view(x.shape))
    with pytest.raises(RuntimeError, match="contiguous"):
        tq_ops.tr(torch.zeros(4, 6)[:, ::2], 1.0, 8, 1, 1)
    with pytest.raises(RuntimeError, match="not implemented"):
        tq_ops.tr(torch.zeros(2, 4, dtype=torch.int32), 1.0, 8, 1, 1)
    with pytest.raises(RuntimeError, match="CUDA"):
        tq_ops.tr(torch.zeros(2, 4, device="meta"), 1.0, 8, 1, 1)


def _errs_restated(x, hist, sfs, bw, k):
    """tq_mse_profile's contract in numpy: per-bin fp32 hist * (x - xh)^2 with xh the oracle's
    TR, summed in fp64 as 256 strided partials and a pairwise tree (csrc/tq_calib.hip)."""
    out = []
    for sf in sfs:
        xh = oracle.tr(x.reshape(-1, 1, 1, 1), sf, bw, 1, k).reshape(-1)
        d = (x - xh).astype(np.float32)
        e = (hist * (d * d)).astype(np.float32).astype(np.float64)
        part = [0.0] * 256
        for p in range(256):  # sequential per partial (acc += e), as the kernel
            acc = 0.0
            for v in e[p::256].tolist():
                acc += v
            part[p] = acc
        w = 128
        while w:
            for t in range(w):
                part[t] += part[t + w]
            w //= 2
        out.append(part[0])
    return np.array(out)


def test_host_mse_profile_matches_restatement():
    rng = np.random.default_rng(5)
    x = torch.linspace(-50, 50, 8192)
    hist = torch.from_numpy(np.maximum(rng.standard_normal(8192) * 40, 0).astype(np.float32))
    sfs_list = torch.linspace(1e-8, 50, 2048).tolist()
    sfs = torch.tensor(sfs_list, dtype=torch.float32)
    errs = tq_native.mse_profile_host(x, hist, sfs, 9, 3)
    pick = list(range(0, 2048, 97)) + [1, 2, 2047]
    exp = _errs_restated(x.numpy(), hist.numpy(), [sfs_list[i] for i in pick], 9, 3)
    np.testing.assert_array_equal(errs.numpy()[pick], exp)
    # tr_layer.mse_profile on a CPU histogram: the host library, first arg-min
    sf = tr_layer.mse_profile(hist, -50, 50, 9, 3)
    assert sf == sfs_list[int(np.argmin(errs.numpy()))]
    sf_o, errs_o = oracle.mse_profile(hist.numpy(), -50, 50, 9, 3)
    np.testing.assert_allclose(errs.numpy(), errs_o, rtol=1e-12)
    assert sf == sf_o


def test_host_ubsan_clean():
    """The host TR op has no undefined shifts/overflows (host UBSan build)."""
    pkg = os.path.join(ROOT, "term-quantization_amd")
    r = subprocess.run(["make", "-s", "-C", pkg, "lib/libtq_host_ubsan.so"], capture_output=True)
    if r.returncode != 0:
        pytest.skip("UBSan runtime unavailable: %s" % r.stderr.decode()[-200:])
    so = os.path.join(pkg, "lib", "libtq_host_ubsan.so")
    code = (
        "import ctypes, numpy as np\n"
        "l = ctypes.CDLL(%r)\n"
        "V, I64, I32, F32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float\n"
        "l.tq_tr_f32_host.argtypes = [V, V, I64, V, F32, I32, I32, I32, I32]\n"
        "l.tq_mse_profile_host.argtypes = [V, V, I64, V, I64, I32, I32, V, I32]\n"
        "x = (np.random.default_rng(0).standard_normal((4, 64, 3)) * 40).astype(np.float32)\n"
        "x[0, :4, 0] = [np.inf, -np.inf, np.nan, 1e38]\n"
        "o = np.empty_like(x); s = (ctypes.c_int64 * 3)(4, 64, 3)\n"
        "for bw, g, k in [(16, 8, 12), (24, 32, 96), (9, 1, 3), (0, 3, 2), (24, 1, 30)]:\n"
        "    for sf in (1e-3, 0.0, float('inf')):\n"
        "        rc = l.tq_tr_f32_host(x.ctypes.data, o.ctypes.data, 3, s, sf, bw, g, k, 2)\n"
        "        assert rc == 0\n"
        "xs = np.linspace(-50, 50, 8192).astype(np.float32); h = np.ones(8192, np.float32)\n"
        "sfs = np.linspace(1e-8, 50, 64).astype(np.float32); e = np.empty(64)\n"
        "assert l.tq_mse_profile_host(xs.ctypes.data, h.ctypes.data, 8192, sfs.ctypes.data, 64,"
        " 24, 24, e.ctypes.data, 2) == 0\n" % so)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    assert b"runtime error" not in r.stderr


def test_layers_on_cpu_use_the_host_tr():
    """TR layers built on CPU: weights through the host TR op (bit-exact vs the oracle), the
    reference composition for the forward, calibration through the host mse_profile."""
    torch.manual_seed(1)
    lin = nn.Linear(650, 40)
    w0 = lin.weight.detach().clone()
    layer = tr_layer.TRLinearLayer(lin, 8, 8, 8, 8, 12)  # 650 % 8 != 0: partial last group
    sf = w0.abs().max().item() / 128
    assert torch.equal(layer.linear.weight.detach(),
                       torch.from_numpy(oracle.tr(w0.numpy(), sf, 8, 8, 12)))
    x = torch.randn(5, 650)
    with torch.no_grad():
        layer(x)
    layer.tracking(False)
    assert not layer.input_quant.tracking and layer.input_quant.sf > 0
    with torch.no_grad():
        assert torch.equal(layer(x), layer.linear(x))  # reference: output on the raw x
    conv = nn.Conv2d(16, 8, 3, padding=1)
    cl = tr_layer.TRConv2dLayer(conv, 9, 3, 9, 8, 12)
    assert cl.mode == "termpair"  # packed for the GPU kernels; a CPU input runs conv(TR(x))
    xc = torch.relu(torch.randn(2, 16, 6, 6))
    with torch.no_grad():
        cl(xc)
    cl.tracking(False)
    with torch.no_grad():
        y = cl(xc)
    xq = torch.from_numpy(oracle.tr(xc.numpy().reshape(1, -1, 1, 1), cl.input_quant.sf, 9, 1,
                                    3)).view(xc.shape)
    assert torch.equal(y, conv(xq))


def test_evaluate_mlp_runs_on_cpu(tmp_path):
    """BASELINE configs[0]: evaluate_mlp.py --synthetic --no-cuda end to end (g=8, k=12),
    plus the published evaluate_mlp.sh:4 point (wb=4, g=16, wt=12, db=dt=6) whose term-pair
    MAC count must match results/mnist-tr.json."""
    import evaluate_mlp
    pub = json.load(open(os.path.join(GOLDEN, "published_results.json")))["mnist-tr.json"]
    out = tmp_path / "r.json"
    res = evaluate_mlp.main(["--synthetic", "--no-cuda", "--wb", "4", "4", "--wt", "12", "12",
                             "--db", "6", "6", "--dt", "6", "6", "--gs", "8", "16",
                             "--out-file", str(out)])
    assert json.load(open(out)) == res
    assert len(res["accs"]) == 2 and all(0.0 <= a <= 100.0 for a in res["accs"])
    assert res["tmacs"][1] == pub["tmacs"][3]
    # g=8, k=12 has no published point; same formula, alpha = k/g twice the g=16 one
    assert res["tmacs"][0] == 2 * pub["tmacs"][3]


@pytest.mark.gpu
def test_evaluate_mlp_runs_on_cpu_in_gpu_run(tmp_path):
    """The same BASELINE configs[0] run (CPU torch, host TR op) inside the -m gpu selection,
    so the round-end GPU-box run records the MNIST MLP config too."""
    test_evaluate_mlp_runs_on_cpu(tmp_path)


def test_lstm_termpair_falls_back_past_the_int32_bound():
    """TRLSTMLayer keeps its term-pair path only while the exact int32 sums cannot wrap
    (sum_k |v_w| << data_bits < 2^31 for both layer-0 weights, as TRConv2dLayer and
    TRLinearLayer check it); at 14-bit weights and activations over K = 650 they can, so the
    layer falls back to the reference composition (library LSTM on TR'd tensors)."""
    torch.manual_seed(0)
    ok = tr_layer.TRLSTMLayer(nn.LSTM(650, 650, 2), 8, 8, 8, 8, 12)
    assert ok.termpair and hasattr(ok, "w_codes_ih") and hasattr(ok, "w_codes_hh")
    lstm = nn.LSTM(650, 650, 2)
    w_hh = lstm.weight_hh_l0.detach().clone()
    big = tr_layer.TRLSTMLayer(lstm, 14, 8, 14, 8, 12)
    assert not big.termpair
    assert not hasattr(big, "w_codes_ih") and not hasattr(big, "w_codes_hh")
    # weights still TR'd (bit-exact vs the oracle); w_sf is the hh scale, as the reference's
    sf = w_hh.abs().max().item() / 2**13
    assert big.w_sf == sf
    assert torch.equal(big.lstm.weight_hh_l0.detach(),
                       torch.from_numpy(oracle.tr(w_hh.numpy(), sf, 14, 8, 12)))
