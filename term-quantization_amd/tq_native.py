"""ctypes binding of libtq_hip.so (include/tq.h) for torch tensors.

This is the only place the Python host layer touches native code.  The libraries are built
in-tree (``make -C term-quantization_amd`` or ``__graft_entry__.build()``) and loaded from
``term-quantization_amd/lib/``: ``libtq_hip.so`` (include/tq.h, the MI355X kernels) for CUDA
tensors and ``libtq_host.so`` (include/tq_host.h, the OpenMP CPU TR op) for CPU tensors.  If the
library a call needs is missing it raises -- there is no PyTorch fallback, and a CUDA tensor
never runs on the host library.

Every call enqueues on torch's current HIP stream of the tensor's device, so the ops order
correctly with surrounding torch work and can be captured into a CUDA/HIP graph.
"""
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# TQ_LIB_PATH: an alternative in-tree build of the same library (tools: ablation builds)
LIB_PATH = os.environ.get("TQ_LIB_PATH") or os.path.join(_HERE, "lib", "libtq_hip.so")
HOST_LIB_PATH = os.path.join(_HERE, "lib", "libtq_host.so")

_lib = None
_host_lib = None
_lock = threading.Lock()

_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_f32 = ctypes.c_float
_f64 = ctypes.c_double
_vp = ctypes.c_void_p

# name -> argtypes (all return int status unless listed in _RESTYPE)
_SIGNATURES = {
    "tq_version": [],
    "tq_last_error": [],
    "tq_sync_faults": [ctypes.POINTER(ctypes.c_uint32)],
    "tq_lstm_seq_workspace_bytes": [_i64, _i64],
    "tq_lstm_seq_f32": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _i64, _vp],
    "tq_lstm_seq2_supported": [_i64, _i64],
    "tq_lstm_seq2_f32": [_vp] * 15 + [_i64, _i64, _i64, _vp],
    "tq_tr_f32": [_vp, _vp, _i64, ctypes.POINTER(_i64), _f32, _i32, _i32, _i32, _vp],
    "tq_tr_f64": [_vp, _vp, _i64, ctypes.POINTER(_i64), _f32, _i32, _i32, _i32, _vp],
    "tq_tr_encode_f32": [_vp, _vp, _vp, _i64, ctypes.POINTER(_i64), _f32, _i32, _i32, _i32,
                         _vp],
    "tq_act_encode_act": [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i32, _vp, _f32, _i32,
                          _i32, _vp, _i64, _i32, _vp],
    "tq_act_encode": [_vp, _i32, _i64, _i64, _i64, _i64, _f32, _i32, _i32, _vp, _i64, _i32,
                      _vp],
    "tq_se_gate_f32": [_vp, _i64, _i64, _vp, _i64, _f64, _vp, _f32, _i32, _i32, _vp, _f64, _vp,
                       _f32, _i32, _i32, _vp, _vp],
    "tq_conv2d_cout_align": [],
    "tq_conv2d_num_configs": [],
    "tq_conv2d_workspace_bytes": [_i64, _i64],
    "tq_conv2d_termpair": [_vp, _i64, _i64, _i64, _i64, _vp, _i64, _i64, _i64, _i64, _i64,
                           _i64, _i64, _i64, _i64, _i64, _f64, _vp, _vp, _i64, _i64, _i32,
                           _vp],
    "tq_mse_profile": [_vp, _vp, _i64, _vp, _i64, _i32, _i32, _vp, _vp],
    "tq_histc_f32": [_vp, _i64, _i64, _f32, _f32, _vp, _vp, _vp],
    "tq_lstm_cell_f32": [_vp, _vp, _vp, _vp, _i64, _i64, _vp],
    "tq_conv2d_termpair_wide": [_vp, _i64, _i64, _i64, _i64, _vp, _i64, _i64, _i64, _i64,
                                _i64, _i64, _i64, _i64, _i64, _i64, _f64, _vp, _vp, _i64, _i64,
                                _i32, _vp],
    "tq_bn_relu_maxpool_encode": [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _i32, _i32, _i32,
                                  _vp, _i64, _i64, _vp, _i64, _f32, _i32, _i32, _i32, _vp,
                                  _i64, _f32, _i32, _i32, _i32, _vp],
    "tq_conv2d_mfma_num_configs": [],
    "tq_dwconv2d_termpair": [_vp, _i64, _i64, _i64, _i64, _i64, _vp, _i64, _i64, _i64, _i64,
                             _i64, _i64, _i64, _i64, _f64, _vp, _vp, _i64, _i64, _i32, _vp],
}

class ConvEpilogue(ctypes.Structure):
    """tq_conv_epilogue (include/tq.h)."""
    _fields_ = [("ch_scale", _vp), ("ch_shift", _vp), ("residual", _vp), ("relu", _i32),
                ("codes_a", _vp), ("cp_a", _i64), ("sf_a", _f32), ("bits_a", _i32),
                ("terms_a", _i32),
                ("codes_b", _vp), ("cp_b", _i64), ("sf_b", _f32), ("bits_b", _i32),
                ("terms_b", _i32),
                ("workspace", _vp), ("workspace_bytes", _i64), ("split_k", _i32),
                ("config", _i32), ("fmt_a", _i32), ("fmt_b", _i32),
                ("ds_codes", _vp), ("ds_h", _i64), ("ds_w", _i64), ("ds_cp", _i64),
                ("ds_stride", _i64), ("ds_w_codes", _vp), ("ds_scale", _vp), ("ds_shift", _vp)]


_SIGNATURES["tq_conv2d_termpair_fused"] = [
    _vp, _i64, _i64, _i64, _i64, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64,
    _i64, _f64, _vp, _vp, _i64, _i64, ctypes.POINTER(ConvEpilogue), _vp]

class DwEpilogue(ctypes.Structure):
    """tq_dw_epilogue (include/tq.h)."""
    _fields_ = [("ch_scale", _vp), ("ch_shift", _vp), ("relu", _i32), ("codes", _vp),
                ("cp", _i64), ("sf", _f32), ("bits", _i32), ("terms", _i32), ("fmt", _i32)]


_SIGNATURES["tq_dwconv2d_termpair_fused"] = [
    _vp, _i64, _i64, _i64, _i64, _i64, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64,
    _vp, _i64, _i64, ctypes.POINTER(DwEpilogue), _vp]

_SIGNATURES["tq_stem_conv_pool_encode"] = [
    _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _i64, _f32, _i32, _i32, _i32,
    _vp, _i64, _f32, _i32, _i32, _i32, _vp, _vp, _vp, _i64, _vp]
_SIGNATURES["tq_stem_workspace_bytes"] = [_i64, _i64, _i64]
_SIGNATURES["tq_conv2d_termpair_f16"] = [
    _vp, _i64, _i64, _i64, _i64, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64,
    _i64, _f64, _vp, _vp, _i64, _i64, _i32, _i32, _i32, ctypes.POINTER(ConvEpilogue), _vp]

# include/tq.h TQ_CODES_*: the code format follows the code tensor's dtype
CODES_I16 = 0
CODES_F16 = 1


def code_format(codes):
    """TQ_CODES_* of a code tensor: int16 -> TQ_CODES_I16, float16 -> TQ_CODES_F16."""
    if codes.dtype == torch.int16:
        return CODES_I16
    if codes.dtype == torch.float16:
        return CODES_F16
    raise RuntimeError("term-pair codes must be int16 or float16 (got %s)" % codes.dtype)


_RESTYPE = {"tq_version": ctypes.c_char_p, "tq_last_error": ctypes.c_char_p,
            "tq_conv2d_cout_align": _i64, "tq_conv2d_num_configs": _i32,
            "tq_conv2d_mfma_num_configs": _i32,
            "tq_conv2d_workspace_bytes": _i64, "tq_lstm_seq_workspace_bytes": _i64}

EXPORTED_SYMBOLS = tuple(_SIGNATURES)


class NativeLibraryMissing(RuntimeError):
    pass


def lib():
    """Load libtq_hip.so once; raise if it has not been built."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise NativeLibraryMissing(
                        "term-quantization HIP library not found at %s; build it with "
                        "`make -C term-quantization_amd` (there is no CPU fallback)" % LIB_PATH)
                l = ctypes.CDLL(LIB_PATH)
                for name, argtypes in _SIGNATURES.items():
                    if os.environ.get("TQ_LIB_PATH") and not hasattr(l, name):
                        continue  # an older A/B build (tools only) may lack newer entries
                    fn = getattr(l, name)
                    fn.argtypes = argtypes
                    fn.restype = _RESTYPE.get(name, ctypes.c_int)
                _lib = l
    return _lib


# include/tq_host.h: name -> argtypes (int status unless in _HOST_RESTYPE)
_HOST_SIGNATURES = {
    "tq_host_version": [],
    "tq_host_last_error": [],
    "tq_tr_f32_host": [_vp, _vp, _i64, ctypes.POINTER(_i64), _f32, _i32, _i32, _i32, _i32],
    "tq_tr_f64_host": [_vp, _vp, _i64, ctypes.POINTER(_i64), _f32, _i32, _i32, _i32, _i32],
    "tq_tr_encode_f32_host": [_vp, _vp, _vp, _i64, ctypes.POINTER(_i64), _f32, _i32, _i32,
                              _i32, _i32],
    "tq_mse_profile_host": [_vp, _vp, _i64, _vp, _i64, _i32, _i32, _vp, _i32],
}
_HOST_RESTYPE = {"tq_host_version": ctypes.c_char_p, "tq_host_last_error": ctypes.c_char_p}
HOST_EXPORTED_SYMBOLS = tuple(_HOST_SIGNATURES)


def host_lib():
    """Load libtq_host.so (the CPU TR op) once; raise if it has not been built."""
    global _host_lib
    if _host_lib is None:
        with _lock:
            if _host_lib is None:
                if not os.path.exists(HOST_LIB_PATH):
                    raise NativeLibraryMissing(
                        "term-quantization host library not found at %s; build it with "
                        "`make -C term-quantization_amd`" % HOST_LIB_PATH)
                l = ctypes.CDLL(HOST_LIB_PATH)
                for name, argtypes in _HOST_SIGNATURES.items():
                    fn = getattr(l, name)
                    fn.argtypes = argtypes
                    fn.restype = _HOST_RESTYPE.get(name, ctypes.c_int)
                _host_lib = l
    return _host_lib


def _check_host(rc):
    if rc != 0:
        raise RuntimeError(host_lib().tq_host_last_error().decode())


def _host_threads():
    return int(torch.get_num_threads())


def tr_into_host(inp, out, sf, bitwidth, group_size, num_keep_terms, codes=None):
    """The TR op on contiguous CPU tensors (tq_tr_*_host); OpenMP with torch's intra-op
    thread count.  ctypes drops the GIL for the call."""
    shape = (_i64 * inp.dim())(*inp.shape)
    nt = _host_threads()
    if codes is not None:
        rc = host_lib().tq_tr_encode_f32_host(_ptr(inp), _ptr(out), _ptr(codes), inp.dim(),
                                              shape, sf, bitwidth, group_size, num_keep_terms,
                                              nt)
    elif inp.dtype == torch.float32:
        rc = host_lib().tq_tr_f32_host(_ptr(inp), _ptr(out), inp.dim(), shape, sf, bitwidth,
                                       group_size, num_keep_terms, nt)
    else:
        rc = host_lib().tq_tr_f64_host(_ptr(inp), _ptr(out), inp.dim(), shape, sf, bitwidth,
                                       group_size, num_keep_terms, nt)
    _check_host(rc)
    return out


def mse_profile_host(x, hist, sfs, bitwidth, num_keep_terms):
    """errs[s] (float64, CPU) for each candidate scale in sfs (tq_mse_profile_host): the same
    values, in the same summation order, as mse_profile on the GPU."""
    errs = torch.empty(sfs.numel(), dtype=torch.float64)
    rc = host_lib().tq_mse_profile_host(_ptr(x), _ptr(hist), x.numel(), _ptr(sfs), sfs.numel(),
                                        int(bitwidth), int(num_keep_terms), _ptr(errs),
                                        _host_threads())
    _check_host(rc)
    return errs


def version():
    return lib().tq_version().decode()


def sync_faults():
    """Bounded in-kernel waits that ran out since the last call (then cleared; synchronous):
    the row-strip conv engine's team syncs, the only bounded spin left (tq_sync_faults); 0 in
    a healthy run."""
    n = ctypes.c_uint32(0)
    _check(lib().tq_sync_faults(ctypes.byref(n)))
    return int(n.value)


_lstm_ws = {}


def lstm_seq_workspace_bytes(batch, hidden):
    """tq_lstm_seq_workspace_bytes: device bytes the recurrence call needs, < 0 if the shape is
    outside its domain."""
    return int(lib().tq_lstm_seq_workspace_bytes(batch, hidden))


def lstm_seq(gx, w_hh, b_hh, h0, c0, out, c_out):
    """A whole LSTM layer's recurrence from one call (tq_lstm_seq_f32: T launches of the fused
    step kernel, h W_hh^T + gates + cell): gx
    [T, B, 4H], w_hh [4H, H], b_hh [4H] or None, h0/c0/c_out [B, H], out [T, B, H], contiguous
    fp32 CUDA tensors; the workspace is cached per (device, B, H)."""
    t, b, h4 = gx.shape
    hid = h4 // 4
    key = (gx.device, b, hid)
    ws = _lstm_ws.get(key)
    if ws is None:
        nb = int(lib().tq_lstm_seq_workspace_bytes(b, hid))
        ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=gx.device)
        _lstm_ws[key] = ws
    with torch.cuda.device(gx.device):
        rc = lib().tq_lstm_seq_f32(_ptr(gx), _ptr(w_hh), _ptr(b_hh), _ptr(h0), _ptr(c0),
                                   _ptr(out), _ptr(c_out), t, b, hid, _ptr(ws), ws.numel(),
                                   _stream(gx))
    _check(rc)
    return out


def lstm_seq2_supported(batch, hidden):
    """tq_lstm_seq2_supported: the two-layer wavefront call covers (batch, hidden)."""
    return bool(lib().tq_lstm_seq2_supported(batch, hidden))


def lstm_seq2(gx0, w_hh0, b_hh0, h00, c00, w_ih1, b_ih1, w_hh1, b_hh1, h01, c01, out0, out1,
              c_out0, c_out1):
    """Two stacked LSTM layers' recurrences in wavefront order (tq_lstm_seq2_f32: steps + 1
    launches, layer 1's input projection inside its steps): gx0 [T, B, 4H] (layer 0's input
    projection incl. b_ih0), weights [4H, H], biases [4H] or None, initial states [B, H],
    out0 / out1 [T, B, H], c_out0 / c_out1 [B, H]; contiguous fp32 CUDA tensors."""
    t, b, h4 = gx0.shape
    with torch.cuda.device(gx0.device):
        rc = lib().tq_lstm_seq2_f32(
            _ptr(gx0), _ptr(w_hh0), _ptr(b_hh0), _ptr(h00), _ptr(c00), _ptr(w_ih1),
            _ptr(b_ih1), _ptr(w_hh1), _ptr(b_hh1), _ptr(h01), _ptr(c01), _ptr(out0),
            _ptr(out1), _ptr(c_out0), _ptr(c_out1), t, b, h4 // 4, _stream(gx0))
    _check(rc)
    return out0, out1


def _check(rc):
    if rc != 0:
        msg = lib().tq_last_error().decode()
        raise RuntimeError(msg)


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def tr_into(inp, out, sf, bitwidth, group_size, num_keep_terms, codes=None):
    """Launch the TR op (tq_tr_f32 / tq_tr_f64 / tq_tr_encode_f32) on contiguous tensors."""
    shape = (_i64 * inp.dim())(*inp.shape)
    with torch.cuda.device(inp.device):
        if codes is not None:
            rc = lib().tq_tr_encode_f32(_ptr(inp), _ptr(out), _ptr(codes), inp.dim(), shape,
                                        sf, bitwidth, group_size, num_keep_terms, _stream(inp))
        elif inp.dtype == torch.float32:
            rc = lib().tq_tr_f32(_ptr(inp), _ptr(out), inp.dim(), shape, sf, bitwidth,
                                 group_size, num_keep_terms, _stream(inp))
        else:
            rc = lib().tq_tr_f64(_ptr(inp), _ptr(out), inp.dim(), shape, sf, bitwidth,
                                 group_size, num_keep_terms, _stream(inp))
    _check(rc)
    return out


def act_encode(x, in_nhwc, sf, bitwidth, num_keep_terms, codes):
    """TR of x into NHWC codes; int16 ``codes`` for the VALU engine, float16 for MFMA."""
    n, c, h, w = x.shape
    fmt = code_format(codes)
    with torch.cuda.device(x.device):
        rc = lib().tq_act_encode(_ptr(x), int(in_nhwc), n, c, h, w, sf, bitwidth,
                                 num_keep_terms, _ptr(codes), codes.shape[-1], fmt, _stream(x))
    _check(rc)
    return codes


def act_code(relu):
    """Epilogue activation code of include/tq.h: False/0 none, True/1 ReLU, 6 ReLU6,
    "swish" swish (EfficientNet)."""
    if relu == "swish":
        return 3
    if relu is None:
        return 0
    return 2 if relu == 6 else int(bool(relu))


def act_encode_act(x, sf, bitwidth, num_keep_terms, codes, act=None, gate=None, out=None,
                   affine=None):
    """codes = TR(gate[n, c] * act(x * scale[c] + shift[c])) (tq_act_encode_act): x fp32
    channels_last [N, C, H, W], ``affine`` None or fp32 (scale, shift) [C] (an eval BN), act
    None / True / 6 / "swish", gate None or fp32 [N, C] (EfficientNet's squeeze-excite
    sigmoid), ``out`` (optional, channels_last like x) receives act(affine(x))."""
    n, c, h, w = x.shape
    if not x.is_contiguous(memory_format=torch.channels_last):
        raise RuntimeError("act_encode_act: x must be channels_last")
    if gate is not None and (gate.dtype != torch.float32 or tuple(gate.shape) != (n, c) or
                             not gate.is_contiguous()):
        raise RuntimeError("act_encode_act: gate must be a contiguous fp32 [N, C] tensor")
    if out is not None and (out.shape != x.shape or
                            not out.is_contiguous(memory_format=torch.channels_last)):
        raise RuntimeError("act_encode_act: out must be channels_last like x")
    with torch.cuda.device(x.device):
        sc, sh = affine if affine is not None else (None, None)
        rc = lib().tq_act_encode_act(_ptr(x), n, c, h, w, _ptr(sc), _ptr(sh), _ptr(gate),
                                     act_code(act), _ptr(out),
                                     sf, bitwidth, num_keep_terms, _ptr(codes), codes.shape[-1],
                                     code_format(codes), _stream(x))
    _check(rc)
    return codes


def se_gate(x_sq, w_r, scale_r, b_r, quant_r, w_e_t, scale_e, b_e, quant_e, gate):
    """EfficientNet squeeze-excite gate in one launch (tq_se_gate_f32): gate [N, C] =
    sigmoid(expand(swish(reduce(x_sq)))) with x_sq fp32 [N, C], int32 weight codes w_r
    [Cse, roundup(C, 8)] and w_e_t [Cse, C] (the expand conv's codes transposed), quant_* =
    (sf, bits, terms) of each conv's input quantizer, scale_* = double(sf_x) * double(sf_w)."""
    n, c = x_sq.shape
    cse = w_r.shape[0]
    for t, shp in ((w_r, (cse, (c + 7) // 8 * 8)), (w_e_t, (cse, c))):
        if t.dtype != torch.int32 or tuple(t.shape) != shp or not t.is_contiguous():
            raise RuntimeError("se_gate: weight codes must be contiguous int32 %s" % (shp,))
    with torch.cuda.device(x_sq.device):
        rc = lib().tq_se_gate_f32(_ptr(x_sq), n, c, _ptr(w_r), cse, float(scale_r), _ptr(b_r),
                                  float(quant_r[0]), int(quant_r[1]), int(quant_r[2]), _ptr(w_e_t),
                                  float(scale_e), _ptr(b_e), float(quant_e[0]),
                                  int(quant_e[1]), int(quant_e[2]), _ptr(gate), _stream(x_sq))
    _check(rc)
    return gate


def conv2d_cout_align():
    return int(lib().tq_conv2d_cout_align())


def conv2d_termpair(codes, w_codes, cout, kh, kw, stride, padding, dilation, scale, bias, out,
                    out_nhwc, kc_steps=0, kc_chunk=-1):
    """Plain term-pair conv.  int16 codes run the VALU engine (tq_conv2d_termpair), float16
    codes the MFMA engine (tq_conv2d_termpair_f16, flush intervals ``kc_steps`` /
    ``kc_chunk``)."""
    n, h, w, cp = codes.shape
    ho, wo = out.shape[2], out.shape[3]
    fmt = code_format(codes)
    if code_format(w_codes) != fmt:
        raise RuntimeError("activation and weight codes must have the same format")
    with torch.cuda.device(codes.device):
        if fmt == CODES_F16:
            rc = lib().tq_conv2d_termpair_f16(
                _ptr(codes), n, h, w, cp, _ptr(w_codes), cout, kh, kw, w_codes.shape[1],
                stride[0], stride[1], padding[0], padding[1], dilation[0], dilation[1],
                float(scale), _ptr(bias), _ptr(out), ho, wo, int(out_nhwc), int(kc_steps),
                int(kc_chunk), None, _stream(codes))
        else:
            rc = lib().tq_conv2d_termpair(_ptr(codes), n, h, w, cp, _ptr(w_codes), cout, kh,
                                          kw, w_codes.shape[1], stride[0], stride[1],
                                          padding[0], padding[1], dilation[0], dilation[1],
                                          float(scale), _ptr(bias), _ptr(out), ho, wo,
                                          int(out_nhwc), _stream(codes))
    _check(rc)
    return out


def conv2d_termpair_wide(codes, w_codes, cout, kh, kw, stride, padding, dilation, scale, bias,
                         out, out_nhwc):
    """Term-pair conv with int32 weight codes (tq_conv2d_termpair_wide): int16 activation
    codes [n, h, w, cp], w_codes int32 [cout, kh*kw*cp]."""
    n, h, w, cp = codes.shape
    ho, wo = out.shape[2], out.shape[3]
    with torch.cuda.device(codes.device):
        rc = lib().tq_conv2d_termpair_wide(
            _ptr(codes), n, h, w, cp, _ptr(w_codes), cout, kh, kw, w_codes.shape[1],
            stride[0], stride[1], padding[0], padding[1], dilation[0], dilation[1],
            float(scale), _ptr(bias), _ptr(out), ho, wo, int(out_nhwc), _stream(codes))
    _check(rc)
    return out


def mse_profile(x, hist, sfs, bitwidth, num_keep_terms):
    """errs[s] (float64) for each candidate scale factor in sfs (tq_mse_profile)."""
    errs = torch.empty(sfs.numel(), dtype=torch.float64, device=x.device)
    with torch.cuda.device(x.device):
        rc = lib().tq_mse_profile(_ptr(x), _ptr(hist), x.numel(), _ptr(sfs), sfs.numel(),
                                  int(bitwidth), int(num_keep_terms), _ptr(errs), _stream(x))
    _check(rc)
    return errs


def lstm_cell(gx, hh, c, h):
    """c <- sigmoid(f) c + sigmoid(i) tanh(g); h = sigmoid(o) tanh(c) for gates = gx + hh
    (tq_lstm_cell_f32); gx, hh [B, 4H], c, h [B, H], contiguous fp32 CUDA tensors."""
    b, hid = c.shape
    with torch.cuda.device(c.device):
        rc = lib().tq_lstm_cell_f32(_ptr(gx), _ptr(hh), _ptr(c), _ptr(h), b, hid, _stream(c))
    _check(rc)
    return h


def histc_accumulate(x, hist, minv, maxv, counts):
    """hist += torch.histc(x, hist.numel(), minv, maxv) with exact counts (tq_histc_f32).
    x: dense fp32 CUDA tensor (any memory format); hist: contiguous fp32 [nbins] on x's device;
    counts: zeroed int64 scratch [nbins] on that device (left zeroed)."""
    with torch.cuda.device(x.device):
        rc = lib().tq_histc_f32(_ptr(x), x.numel(), hist.numel(), float(minv), float(maxv),
                                _ptr(counts), _ptr(hist), _stream(x))
    _check(rc)
    return hist


def conv2d_termpair_fused(codes, w_codes, cout, kh, kw, stride, padding, dilation, ho, wo,
                          out=None, ch_scale=None, ch_shift=None, residual=None, relu=False,
                          codes_a=None, quant_a=None, codes_b=None, quant_b=None,
                          workspace=None, split_k=0, config=0, kc_steps=0, kc_chunk=-1,
                          downsample=None):
    """Term-pair conv with the fused epilogue of tq_conv2d_termpair_fused (channels_last).
    quant_a/_b = (sf, bits, terms) of the layer consuming codes_a/_b, whose dtype (int16 /
    float16) is that layer's code format.  ``workspace`` (int32, >= n*ho*wo*cout elements)
    lets the VALU kernel split the K loop over workgroups.  float16 input codes run the MFMA
    engine (tq_conv2d_termpair_f16) with flush interval ``kc_steps``.  ``downsample`` =
    (codes, w_codes, stride, scale, shift): the fused 1x1 downsample phase whose identity
    replaces ``residual`` (tq_conv_epilogue.ds_*)."""
    n, h, w, cp = codes.shape
    fmt = code_format(codes)
    if code_format(w_codes) != fmt:
        raise RuntimeError("activation and weight codes must have the same format")
    epi = ConvEpilogue()
    epi.ch_scale, epi.ch_shift = _ptr(ch_scale), _ptr(ch_shift)
    epi.residual, epi.relu = _ptr(residual), act_code(relu)
    if codes_a is not None:
        epi.codes_a, epi.cp_a = _ptr(codes_a), codes_a.shape[-1]
        epi.sf_a, epi.bits_a, epi.terms_a = float(quant_a[0]), int(quant_a[1]), int(quant_a[2])
        epi.fmt_a = code_format(codes_a)
    if codes_b is not None:
        epi.codes_b, epi.cp_b = _ptr(codes_b), codes_b.shape[-1]
        epi.sf_b, epi.bits_b, epi.terms_b = float(quant_b[0]), int(quant_b[1]), int(quant_b[2])
        epi.fmt_b = code_format(codes_b)
    if not config and fmt == CODES_F16 and os.environ.get("TQ_MFMA_CONFIG"):
        config = int(os.environ["TQ_MFMA_CONFIG"])  # A/B of MFMA tile configs (tools only)
    epi.workspace, epi.split_k, epi.config = _ptr(workspace), int(split_k), int(config)
    epi.workspace_bytes = workspace.numel() * workspace.element_size() if workspace is not None \
        else 0
    if downsample is not None:
        dcodes, dw, dstride, dscale, dshift = downsample
        epi.ds_codes, epi.ds_w_codes = _ptr(dcodes), _ptr(dw)
        epi.ds_h, epi.ds_w, epi.ds_cp = dcodes.shape[1], dcodes.shape[2], dcodes.shape[3]
        epi.ds_stride = int(dstride)
        epi.ds_scale, epi.ds_shift = _ptr(dscale), _ptr(dshift)
    with torch.cuda.device(codes.device):
        if fmt == CODES_F16:
            rc = lib().tq_conv2d_termpair_f16(
                _ptr(codes), n, h, w, cp, _ptr(w_codes), cout, kh, kw, w_codes.shape[1],
                stride[0], stride[1], padding[0], padding[1], dilation[0], dilation[1], 0.0,
                None, _ptr(out), ho, wo, 1, int(kc_steps), int(kc_chunk), ctypes.byref(epi),
                _stream(codes))
        else:
            rc = lib().tq_conv2d_termpair_fused(
                _ptr(codes), n, h, w, cp, _ptr(w_codes), cout, kh, kw, w_codes.shape[1],
                stride[0], stride[1], padding[0], padding[1], dilation[0], dilation[1], 0.0,
                None, _ptr(out), ho, wo, ctypes.byref(epi), _stream(codes))
    _check(rc)


def dwconv2d_termpair(codes, c, w_codes, kh, kw, stride, pad_tl, dilation, scale, bias, out,
                      out_nhwc):
    """Depthwise term-pair conv (tq_dwconv2d_termpair); w_codes int32 [kh*kw, cp]."""
    n, h, w, cp = codes.shape
    ho, wo = out.shape[2], out.shape[3]
    with torch.cuda.device(codes.device):
        rc = lib().tq_dwconv2d_termpair(_ptr(codes), n, h, w, c, cp, _ptr(w_codes), kh, kw,
                                        stride[0], stride[1], pad_tl[0], pad_tl[1],
                                        dilation[0], dilation[1], float(scale), _ptr(bias),
                                        _ptr(out), ho, wo, int(out_nhwc), _stream(codes))
    _check(rc)
    return out


def dwconv2d_termpair_fused(codes, c, w_codes, kh, kw, stride, pad_tl, dilation, ho, wo,
                            ch_scale, ch_shift, relu, out=None, next_codes=None, quant=None):
    """Depthwise term-pair conv with the fused BN / ReLU(6) / next-layer-codes epilogue
    (tq_dwconv2d_termpair_fused), channels_last; relu 0, 1, 6 or "swish"."""
    n, h, w, cp = codes.shape
    epi = DwEpilogue()
    epi.ch_scale, epi.ch_shift = _ptr(ch_scale), _ptr(ch_shift)
    epi.relu = act_code(relu)
    if next_codes is not None:
        epi.codes, epi.cp = _ptr(next_codes), next_codes.shape[-1]
        epi.sf, epi.bits, epi.terms = float(quant[0]), int(quant[1]), int(quant[2])
        epi.fmt = code_format(next_codes)
    with torch.cuda.device(codes.device):
        rc = lib().tq_dwconv2d_termpair_fused(
            _ptr(codes), n, h, w, c, cp, _ptr(w_codes), kh, kw, stride[0], stride[1],
            pad_tl[0], pad_tl[1], dilation[0], dilation[1], _ptr(out), ho, wo,
            ctypes.byref(epi), _stream(codes))
    _check(rc)
    return out


def conv2d_workspace(pixels, cout, device):
    """Scratch for the K-split schedules of tq_conv2d_termpair_fused (int32 tensor)."""
    with torch.cuda.device(device):
        nbytes = int(lib().tq_conv2d_workspace_bytes(int(pixels), int(cout)))
    return torch.empty((nbytes + 3) // 4, dtype=torch.int32, device=device)


def stem_workspace(n, h, w, device):
    """Scratch of the fused stem's exact fix-up (uint8 tensor, tq_stem_workspace_bytes)."""
    nbytes = int(lib().tq_stem_workspace_bytes(int(n), int(h), int(w)))
    if nbytes < 0:
        raise ValueError("stem_workspace: invalid image size %dx%dx%d" % (n, h, w))
    return torch.empty(nbytes, dtype=torch.uint8, device=device)


def stem_conv_pool_encode(x, w_split, scale, shift, out, codes_a=None, quant_a=None,
                          codes_b=None, quant_b=None, exact=None, workspace=None):
    """relu(maxpool(bn(conv7x7s2(x)))) of a ResNet stem into ``out`` plus next layers' codes
    (tq_stem_conv_pool_encode); x fp32 channels_last [N, 3, H, W], w_split from
    tq_ops.pack_stem_weight.  ``exact`` = (w64, wbound) from tq_ops.pack_stem_exact turns on
    the exact fix-up of near-midpoint outputs (workspace: stem_workspace, allocated here when
    None); without it the split-fp16 conv's result stands."""
    n, c, h, w = x.shape
    ho, wo = out.shape[2], out.shape[3]
    qa = quant_a or (0.0, 0, 0)
    qb = quant_b or (0.0, 0, 0)
    w64 = wbound = None
    if exact is not None:
        w64, wbound = exact
        if workspace is None:
            workspace = stem_workspace(n, h, w, x.device)
    with torch.cuda.device(x.device):
        rc = lib().tq_stem_conv_pool_encode(
            _ptr(x), n, h, w, _ptr(w_split), _ptr(scale), _ptr(shift), _ptr(out), ho, wo,
            _ptr(codes_a), codes_a.shape[-1] if codes_a is not None else 0, float(qa[0]),
            int(qa[1]), int(qa[2]), code_format(codes_a) if codes_a is not None else 0,
            _ptr(codes_b), codes_b.shape[-1] if codes_b is not None else 0, float(qb[0]),
            int(qb[1]), int(qb[2]), code_format(codes_b) if codes_b is not None else 0,
            _ptr(w64), _ptr(wbound), _ptr(workspace if exact is not None else None),
            workspace.numel() if (exact is not None) else 0, _stream(x))
    _check(rc)
    return out


def bn_relu_maxpool_encode(x, scale, shift, k, stride, pad, out, codes_a=None, quant_a=None,
                           codes_b=None, quant_b=None):
    """relu(maxpool(bn(x))) into ``out`` plus next layers' codes (channels_last fp32)."""
    n, c, h, w = x.shape
    ho, wo = out.shape[2], out.shape[3]
    qa = quant_a or (0.0, 0, 0)
    qb = quant_b or (0.0, 0, 0)
    with torch.cuda.device(x.device):
        rc = lib().tq_bn_relu_maxpool_encode(
            _ptr(x), n, h, w, c, _ptr(scale), _ptr(shift), k, stride, pad, _ptr(out), ho, wo,
            _ptr(codes_a), codes_a.shape[-1] if codes_a is not None else 0, float(qa[0]),
            int(qa[1]), int(qa[2]), code_format(codes_a) if codes_a is not None else 0,
            _ptr(codes_b), codes_b.shape[-1] if codes_b is not None else 0, float(qb[0]),
            int(qb[1]), int(qb[2]), code_format(codes_b) if codes_b is not None else 0,
            _stream(x))
    _check(rc)
    return out
