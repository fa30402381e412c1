"""CPU oracle for the term-revealing (TR) path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker (or the timed CPU baseline).  The product path
(``term-quantization_amd/``) never imports it.

It wraps ``liboracle.so`` (``oracle/tr_oracle.c``, a literal C restatement of
``kernels/tr_cuda_kernel.cu``) with numpy, and restates the few Python-level reference
algorithms the path needs (``tr_layer.mse_profile``, the HESE term count behind
``tr_layer.compute_compressed_hese``, the term-pair MAC formula of ``profile_model.py``).
"""
import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build():
    """Compile liboracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE, "liboracle.so"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        l = ctypes.CDLL(_LIB_PATH)
        i64p = ctypes.POINTER(ctypes.c_int64)
        for name, ptr in (("oracle_tr_f32", ctypes.c_float), ("oracle_tr_f64", ctypes.c_double)):
            fn = getattr(l, name)
            fn.restype = ctypes.c_int
            fn.argtypes = [ctypes.POINTER(ptr), ctypes.POINTER(ptr), ctypes.c_int64, i64p,
                           ctypes.c_float, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
        l.oracle_hese_terms.restype = ctypes.c_int
        l.oracle_hese_terms.argtypes = [ctypes.c_int32, ctypes.c_int32,
                                        ctypes.POINTER(ctypes.c_int32)]
        _lib = l
    return _lib


def tr(x, sf, bitwidth, group_size, num_keep_terms):
    """Reference ``tr_cuda.tr`` semantics on a numpy array (float32 or float64).

    Follows kernels/tr_cuda_kernel.cu:58-160 serially; ``sf`` is narrowed to float32 like the
    pybind boundary (kernels/tr_cuda.cpp:20)."""
    x = np.ascontiguousarray(x)
    if x.dtype == np.float32:
        fn, ct = lib().oracle_tr_f32, ctypes.c_float
    elif x.dtype == np.float64:
        fn, ct = lib().oracle_tr_f64, ctypes.c_double
    else:
        raise TypeError("oracle.tr: float32/float64 only")
    out = np.empty_like(x)
    shape = (ctypes.c_int64 * x.ndim)(*x.shape)
    rc = fn(x.ctypes.data_as(ctypes.POINTER(ct)), out.ctypes.data_as(ctypes.POINTER(ct)),
            x.ndim, shape, float(np.float32(sf)), int(bitwidth), int(group_size),
            int(num_keep_terms))
    if rc != 0:
        raise ValueError("oracle.tr: unsupported arguments (rc=%d)" % rc)
    return out


def hese_terms(q):
    """HESE term list of integer q (|q| < 2^24), most significant first, signed like
    bit_utils.hese (bit_utils.py:10-44) and hese_encode (tr_cuda_kernel.cu:14-56)."""
    buf = (ctypes.c_int32 * 64)()
    n = lib().oracle_hese_terms(abs(int(q)), -1 if q < 0 else 1, buf)
    return [int(buf[i]) for i in range(n)]


def hese_masks(qs):
    """(pos, neg) uint32 bitmasks of the HESE terms of each non-negative q, via the oracle's
    literal encoder (the golden fixtures store the same form)."""
    qs = np.asarray(qs, dtype=np.int64)
    pos = np.zeros(qs.shape, np.uint32)
    neg = np.zeros(qs.shape, np.uint32)
    for i, q in enumerate(qs.reshape(-1).tolist()):
        p = n = 0
        for t in hese_terms(q):
            e = abs(t).bit_length() - 1
            if t > 0:
                p |= 1 << e
            else:
                n |= 1 << e
        pos.reshape(-1)[i] = p
        neg.reshape(-1)[i] = n
    return pos, neg


def hese_py(number):
    """Pure-Python restatement of bit_utils.hese (bit_utils.py:10-44): the bit windows
    (b[i+1], b[i], b[i-1]) scanned from the top bit down -- 010 -> sign 2^i (and skip bit
    i-1), 011 -> sign 2^(i+1), 110 -> -sign 2^i -- on Python ints instead of the reference's
    binary strings.  BASELINE C1's single-core baseline (bench.py cpu_baseline)."""
    sign = -1 if number < 0 else 1
    q = -number if number < 0 else number
    out = []
    i = q.bit_length() - 1
    while i >= 0:
        if (q >> i) & 1:
            above = (q >> (i + 1)) & 1
            below = (q >> (i - 1)) & 1 if i > 0 else 0
            if not above:
                if below:
                    out.append(sign * (1 << (i + 1)))
                else:
                    out.append(sign * (1 << i))
                    i -= 1
            elif not below:
                out.append(-sign * (1 << i))
        i -= 1
    return out


def tr_py(x, sf, bitwidth, group_size, num_keep_terms):
    """Pure-Python restatement of the whole tr() on a flat float32 vector grouped by
    consecutive elements (a (1, C) tensor): quantize as tr_cuda_kernel.cu:21-23 (fp32 |x| / sf,
    + 0.5 in double, truncate, clamp to 2^b - 1), hese_py terms, the greedy per-group top-k of
    :92-116 (largest |term| first, the lowest index on ties) and the fp32 rescale of :119-123.
    BASELINE C2's single-core baseline; checked against ``tr`` (the C restatement)."""
    x = np.asarray(x, dtype=np.float32).reshape(-1)
    sf32 = np.float32(sf)
    maxv = (1 << bitwidth) - 1
    out = np.zeros_like(x)
    for g0 in range(0, x.size, group_size):
        terms = []
        for v in x[g0:g0 + group_size]:
            t = float(np.float32(abs(v)) / sf32) + 0.5
            q = min(int(t) if t == t else 0, maxv)
            terms.append(hese_py(-q if v < 0 else q))
        idx = [0] * len(terms)
        for _ in range(num_keep_terms):
            best, bj = 0, 0
            for j, tj in enumerate(terms):
                if idx[j] < len(tj) and abs(tj[idx[j]]) > abs(best):
                    best, bj = tj[idx[j]], j
            if best == 0:
                break
            out[g0 + bj] += np.float32(best)
            idx[bj] += 1
        out[g0:g0 + group_size] *= sf32
    return out


def tr_layer_hese_len(q):
    """len(tr_layer.hese(q)) (tr_layer.py:9-41): runs of ones cost 2 terms, lone ones 1."""
    q = abs(int(q))
    runs = bin(q & ~(q << 1)).count("1")
    singles = bin(q & ~(q << 1) & ~(q >> 1)).count("1")
    return 2 * runs - singles


def mse_profile(hist, minv, maxv, bit_width, terms):
    """tr_layer.mse_profile (tr_layer.py:43-54) on the CPU: 2048 sf candidates over the
    histogram grid, weighted squared error, first arg-min.  The per-bin term
    hist * (x - xh)**2 is formed in float32 like the reference's torch expression; the sum
    over bins is float64 (the reference's fp32 reduction order is torch-internal)."""
    import torch
    x = torch.linspace(minv, maxv, len(hist)).numpy()
    sfs = torch.linspace(1e-8, maxv, 2048).tolist()
    h = np.asarray(hist, dtype=np.float32)
    errs = []
    for sf in sfs:
        xh = tr(x.reshape(-1, 1, 1, 1), sf, bit_width, 1, terms).reshape(-1)
        d = (x - xh).astype(np.float32)
        e = (h * (d * d)).astype(np.float32)
        errs.append(float(e.astype(np.float64).sum()))
    return sfs[int(np.argmin(np.asarray(errs)))], np.asarray(errs)


def histc(x, nbins, minv, maxv):
    """torch.histc(x, nbins, minv, maxv) as the reference's tracking step calls it
    (tr_layer.py:91-94), restated in numpy float32 arithmetic: elements outside [minv, maxv]
    and NaN are skipped, bin = trunc(fp32(fp32(x - minv) * nbins) / (maxv - minv)), bin ==
    nbins goes to the last bin.  Exact int64 counts.  Pinned against torch.histc itself
    (CPU in tests/test_oracle.py, GPU in tests/test_gpu_calib.py)."""
    x = np.asarray(x, dtype=np.float32).reshape(-1)
    lo, hi = np.float32(minv), np.float32(maxv)
    x = x[(x >= lo) & (x <= hi)]
    with np.errstate(over="ignore", invalid="ignore"):
        b = ((x - lo) * np.float32(nbins)) / np.float32(hi - lo)
    b = np.trunc(b).astype(np.int64)
    b[b == nbins] = nbins - 1
    return np.bincount(b, minlength=nbins).astype(np.int64)


def term_pair_macs_conv(out_numel, in_channels, groups, kh, kw, num_terms, weight_bits,
                        group_size, data_terms, data_bits):
    """profile_model.tr_conv2d_ops (profile_model.py:8-26) before the int() truncation."""
    total = out_numel * (in_channels // groups * kh * kw)
    weight_terms = min(num_terms, weight_bits) if group_size == 1 else num_terms
    dterms = min(data_terms, data_bits)
    alpha = weight_terms / group_size
    return dterms * alpha * total


def ceil_log2(n):
    return math.ceil(math.log2(n))
