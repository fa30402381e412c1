"""The C-ABI library (include/tq.h) builds, loads and validates arguments -- CPU-only.

No kernel is launched here (there is no GPU in the build container); every call below is
rejected by argument validation before any HIP runtime call."""
import ctypes
import os
import re

import pytest
import torch

import tq_native
import tq_ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "tq.h")).read()
    return sorted(set(re.findall(r"\b(tq_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = tq_native.lib()
    declared = _declared_symbols()
    assert declared, "no declarations parsed from include/tq.h"
    for name in declared:
        assert hasattr(lib, name), name
    # the Python binding covers exactly the header
    assert sorted(tq_native.EXPORTED_SYMBOLS) == declared


def test_library_is_gfx950_code_object():
    data = open(tq_native.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version_and_error_channel():
    assert tq_native.version().startswith("tq-hip")
    lib = tq_native.lib()
    shape = (ctypes.c_int64 * 1)(4)
    rc = lib.tq_tr_f32(None, None, 1, shape, 1.0, 8, 1, 1, None)
    assert rc == 1
    assert b"at least 2 dimensions" in lib.tq_last_error()


@pytest.mark.parametrize("args,code,msg", [
    (dict(bw=25), 2, b"bitwidth"),
    (dict(bw=-1), 2, b"bitwidth"),
    (dict(g=0), 1, b"group_size"),
    (dict(g=33), 1, b"group_size"),
    (dict(sf=-1.0), 1, b"sf"),
    (dict(sf=float("nan")), 1, b"sf"),
])
def test_tr_argument_validation(args, code, msg):
    lib = tq_native.lib()
    shape = (ctypes.c_int64 * 2)(4, 8)
    p = dict(bw=8, g=1, sf=1.0)
    p.update(args)
    rc = lib.tq_tr_f32(None, None, 2, shape, p["sf"], p["bw"], p["g"], 1, None)
    assert rc == code
    assert msg in lib.tq_last_error()


def test_conv_argument_validation():
    lib = tq_native.lib()
    rc = lib.tq_conv2d_termpair(None, 1, 8, 8, 12, None, 4, 3, 3, 128, 1, 1, 1, 1, 1, 1, 1.0,
                                None, None, 8, 8, 0, None)
    assert rc == 1 and b"cp" in lib.tq_last_error()
    rc = lib.tq_conv2d_termpair(None, 1, 8, 8, 16, None, 4, 3, 3, 100, 1, 1, 1, 1, 1, 1, 1.0,
                                None, None, 8, 8, 0, None)
    assert rc == 1 and b"kp" in lib.tq_last_error()
    rc = lib.tq_conv2d_termpair(None, 1, 8, 8, 16, None, 4, 3, 3, 160, 1, 1, 1, 1, 1, 1, 1.0,
                                None, None, 7, 8, 0, None)
    assert rc == 1 and b"output size" in lib.tq_last_error()
    assert tq_native.conv2d_cout_align() == 128


def test_act_encode_rejects_wide_codes():
    lib = tq_native.lib()
    rc = lib.tq_act_encode(None, 1, 1, 8, 2, 2, 1.0, 16, 3, None, 8, 0, None)
    assert rc == 2 and b"bitwidth" in lib.tq_last_error()
    # fp16 codes are exact only up to 11 bits
    rc = lib.tq_act_encode(None, 1, 1, 8, 2, 2, 1.0, 12, 3, None, 8, 1, None)
    assert rc == 2 and b"fp16" in lib.tq_last_error()
    rc = lib.tq_act_encode(None, 1, 1, 8, 2, 2, 1.0, 9, 3, None, 8, 7, None)
    assert rc == 1 and b"format" in lib.tq_last_error()


def test_conv_f16_argument_validation():
    lib = tq_native.lib()
    # kp must be a multiple of 64 for the MFMA engine
    rc = lib.tq_conv2d_termpair_f16(None, 1, 8, 8, 16, None, 4, 3, 3, 160, 1, 1, 1, 1, 1, 1,
                                    1.0, None, None, 8, 8, 1, 0, -1, None, None)
    assert rc == 1 and b"64" in lib.tq_last_error()
    rc = lib.tq_conv2d_termpair_f16(None, 1, 8, 8, 16, None, 4, 3, 3, 192, 1, 1, 1, 1, 1, 1,
                                    1.0, None, None, 8, 8, 1, -1, -1, None, None)
    assert rc == 1 and b"kc_steps" in lib.tq_last_error()
    epi = tq_native.ConvEpilogue()
    epi.split_k = 2
    out = ctypes.c_void_p(16)
    rc = lib.tq_conv2d_termpair_f16(None, 1, 8, 8, 16, None, 4, 3, 3, 192, 1, 1, 1, 1, 1, 1,
                                    1.0, None, out, 8, 8, 1, 0, -1, ctypes.byref(epi), None)
    assert rc == 2 and b"split" in lib.tq_last_error()
    assert lib.tq_conv2d_mfma_num_configs() >= 1


def test_ops_reject_other_devices_like_the_reference():
    # CPU tensors run on the host library (tests/test_host_tr.py); anything else is refused
    with pytest.raises(RuntimeError, match="CUDA"):
        tq_ops.tr(torch.zeros(2, 4, device="meta"), 1.0, 8, 1, 1)
    with pytest.raises(RuntimeError, match="CUDA"):
        tq_ops.tr_elementwise(torch.zeros(2, 4, device="meta"), 1.0, 8, 1)


def test_histc_argument_validation():
    lib = tq_native.lib()
    buf = 16  # a fake, aligned, non-null address: every call below fails validation first
    assert lib.tq_histc_f32(buf, 8, 0, -50.0, 50.0, buf, buf, None) == 1
    assert b"nbins" in lib.tq_last_error()
    assert lib.tq_histc_f32(buf, 8, 8192, 50.0, 50.0, buf, buf, None) == 1
    assert b"min < max" in lib.tq_last_error()
    assert lib.tq_histc_f32(buf, 8, 8192, -50.0, 50.0, None, buf, None) == 1
    assert b"null" in lib.tq_last_error()
    assert lib.tq_histc_f32(18, 8, 8192, -50.0, 50.0, buf, buf, None) == 1
    assert b"aligned" in lib.tq_last_error()


def test_conv_f16_fused_downsample_validation():
    lib = tq_native.lib()
    out = ctypes.c_void_p(16)
    args = (None, 2, 8, 8, 64, None, 64, 3, 3, 576, 1, 1, 1, 1, 1, 1, 1.0, None, out, 8, 8, 1,
            0, -1)

    def run(**kw):
        epi = tq_native.ConvEpilogue()
        epi.ds_codes, epi.ds_w_codes, epi.ds_scale, epi.ds_shift = 16, 16, 16, 16
        epi.ds_h, epi.ds_w, epi.ds_cp, epi.ds_stride = 16, 16, 64, 2
        for k, v in kw.items():
            setattr(epi, k, v)
        return lib.tq_conv2d_termpair_f16(*args, ctypes.byref(epi), None)

    assert run(residual=16) == 1 and b"replaces the residual" in lib.tq_last_error()
    assert run(ds_w_codes=None) == 1 and b"weights" in lib.tq_last_error()
    assert run(ds_cp=32) == 1 and b"shape" in lib.tq_last_error()
    assert run(ds_h=14) == 1 and b"size mismatch" in lib.tq_last_error()
    assert run(ds_codes=24) == 1 and b"aligned" in lib.tq_last_error()
    assert run(split_k=-1) == 2 and b"data-parallel" in lib.tq_last_error()
    epi = tq_native.ConvEpilogue()
    epi.ds_codes = 16
    rc = lib.tq_conv2d_termpair_fused(None, 2, 8, 8, 64, None, 64, 3, 3, 576, 1, 1, 1, 1, 1, 1,
                                      1.0, None, out, 8, 8, ctypes.byref(epi), None)
    assert rc == 2 and b"MFMA" in lib.tq_last_error()


def test_lstm_cell_argument_validation():
    lib = tq_native.lib()
    assert lib.tq_lstm_cell_f32(None, None, None, None, 2, 3, None) == 1
    assert b"null" in lib.tq_last_error()
    assert lib.tq_lstm_cell_f32(None, None, None, None, -1, 3, None) == 1
    assert lib.tq_lstm_cell_f32(None, None, None, None, 0, 3, None) == 0  # nothing to do


def test_swish_epilogue_and_act_encode_act_validation():
    """relu 3 (swish, EfficientNet) is accepted by the fp16 entry for the direct engine's
    shapes only, never by the VALU entry; tq_act_encode_act validates act and sf."""
    lib = tq_native.lib()
    out = ctypes.c_void_p(16)
    epi = tq_native.ConvEpilogue()
    epi.relu = 4
    rc = lib.tq_conv2d_termpair_f16(None, 1, 8, 8, 64, None, 64, 1, 1, 64, 1, 1, 0, 0, 1, 1,
                                    1.0, None, out, 8, 8, 1, 0, -1, ctypes.byref(epi), None)
    assert rc == 1 and b"relu" in lib.tq_last_error()
    epi.relu = 3
    rc = lib.tq_conv2d_termpair_f16(None, 1, 8, 8, 16, None, 64, 3, 3, 192, 1, 1, 1, 1, 1, 1,
                                    1.0, None, out, 8, 8, 1, 0, -1, ctypes.byref(epi), None)
    assert rc == 2 and b"swish" in lib.tq_last_error()
    rc = lib.tq_conv2d_termpair_fused(None, 1, 8, 8, 64, None, 64, 1, 1, 64, 1, 1, 0, 0, 1, 1,
                                      1.0, None, out, 8, 8, ctypes.byref(epi), None)
    assert rc == 2 and b"swish" in lib.tq_last_error()
    buf = ctypes.c_void_p(64)
    assert lib.tq_act_encode_act(buf, 1, 8, 2, 2, None, None, None, 4, None, 0.1, 9, 3, buf,
                                 8, 1, None) == 1
    assert b"act" in lib.tq_last_error()
    assert lib.tq_act_encode_act(buf, 1, 8, 2, 2, buf, None, None, 2, None, 0.1, 9, 3, buf,
                                 8, 1, None) == 1
    assert b"together" in lib.tq_last_error()
    assert lib.tq_act_encode_act(buf, 1, 8, 2, 2, None, None, None, 3, None, 0.0, 9, 3, buf,
                                 8, 1, None) == 1
    assert b"sf" in lib.tq_last_error()
    assert tq_native.act_code("swish") == 3 and tq_native.act_code(6) == 2


def test_dwconv_fused_requires_the_epilogue_affine():
    """tq_dwconv2d_termpair_fused has no scale/bias of its own: an epilogue without
    ch_scale/ch_shift is rejected (it would otherwise return acc * 0 + 0 everywhere)."""
    lib = tq_native.lib()
    buf = torch.zeros(1 << 16, dtype=torch.float32)
    p = buf.data_ptr()
    epi = tq_native.DwEpilogue(ch_scale=None, ch_shift=None, relu=1, codes=None, cp=16,
                               sf=1.0, bits=8, terms=3, fmt=0)
    rc = lib.tq_dwconv2d_termpair_fused(p, 1, 8, 8, 16, 16, p, 3, 3, 1, 1, 1, 1, 1, 1, p, 8, 8,
                                        ctypes.byref(epi), None)
    assert rc == 1 and b"ch_scale" in lib.tq_last_error()


def test_fused_conv_code_rows_must_be_roundup_cout():
    """Epilogue code targets need cp == roundup(cout, 8): the kernels zero the pad channels
    [cout, cp) only up to the next multiple of 8, so wider rows would keep stale codes."""
    lib = tq_native.lib()
    buf = torch.zeros(1 << 16, dtype=torch.float32)
    p = buf.data_ptr()
    # (only rejected calls here: an accepted one would launch a kernel on host pointers)
    for cp_a in (24, 8, 32):
        epi = tq_native.ConvEpilogue(relu=1, codes_a=p, cp_a=cp_a, sf_a=1.0, bits_a=9,
                                     terms_a=3, fmt_a=1)
        rc = lib.tq_conv2d_termpair_fused(p, 1, 8, 8, 16, p, 12, 3, 3, 192, 1, 1, 1, 1, 1, 1,
                                          1.0, None, p, 8, 8, ctypes.byref(epi), None)
        err = lib.tq_last_error()
        assert rc == 1 and b"roundup(cout, 8)" in err, err


def test_lstm_seq_argument_validation():
    """tq_lstm_seq_f32 rejects sizes outside its domain and a short workspace before any
    launch."""
    lib = tq_native.lib()
    buf = torch.zeros(1 << 16, dtype=torch.float32)
    p = buf.data_ptr()
    rc = lib.tq_lstm_seq_f32(p, p, None, p, p, p, p, 35, 10, 1100, p, 1 << 20, None)
    assert rc == 2 and b"hidden <= 1024" in lib.tq_last_error()
    rc = lib.tq_lstm_seq_f32(p, p, None, p, p, p, p, 35, 100, 650, p, 1 << 20, None)
    assert rc == 2 and b"LDS" in lib.tq_last_error()
    assert tq_native.lstm_seq_workspace_bytes(10, 650) == 0
    assert tq_native.lstm_seq_workspace_bytes(100, 650) < 0
    need = lib.tq_lstm_seq_workspace_bytes(10, 650)
    assert need == 0
    rc = lib.tq_lstm_seq_f32(p, p, None, p, p, p, p, 35, 10, 650, p, need - 8, None)
    assert rc == 1 and b"workspace" in lib.tq_last_error()
    rc = lib.tq_lstm_seq_f32(p, p, None, None, p, p, p, 35, 10, 650, p, need, None)
    assert rc == 1 and b"null" in lib.tq_last_error()
    q = p + 4096
    rc = lib.tq_lstm_seq_f32(p, p, None, p, q, p + 8192, q, 35, 10, 650, None, 0, None)
    assert rc == 1 and b"alias" in lib.tq_last_error()


def test_lstm_seq2_argument_validation():
    """tq_lstm_seq2_f32 rejects shapes outside its domain, null pointers and aliased outputs
    before any launch."""
    lib = tq_native.lib()
    buf = torch.zeros(1 << 16, dtype=torch.float32)
    p = buf.data_ptr()
    ptrs = [p + 256 * i for i in range(15)]
    assert tq_native.lstm_seq2_supported(10, 650)
    assert not tq_native.lstm_seq2_supported(10, 1100)
    assert not tq_native.lstm_seq2_supported(100, 650)
    rc = lib.tq_lstm_seq2_f32(*ptrs, 35, 10, 1100, None)
    assert rc == 2 and b"hidden <= 1024" in lib.tq_last_error()
    bad = list(ptrs)
    bad[3] = None  # h00
    rc = lib.tq_lstm_seq2_f32(*bad, 35, 10, 650, None)
    assert rc == 1 and b"null" in lib.tq_last_error()
    bad = list(ptrs)
    bad[11] = bad[3]  # out0 aliases h00
    rc = lib.tq_lstm_seq2_f32(*bad, 35, 10, 650, None)
    assert rc == 1 and b"alias" in lib.tq_last_error()
    bad = list(ptrs)
    bad[14] = bad[13]  # c_out1 aliases c_out0
    rc = lib.tq_lstm_seq2_f32(*bad, 35, 10, 650, None)
    assert rc == 1 and b"alias" in lib.tq_last_error()
    assert lib.tq_lstm_seq2_f32(*ptrs, 0, 10, 650, None) == 0  # empty: no launch


def test_se_gate_argument_validation():
    """tq_se_gate_f32 rejects bad shapes, null buffers, wide activations and channel counts
    past one workgroup's LDS before any launch; n = 0 is a no-op."""
    lib = tq_native.lib()
    buf = torch.zeros(1 << 12, dtype=torch.float32)
    p = buf.data_ptr()
    args = lambda n, c, cse, br=9, be=9, xp=p: (xp, n, c, p, cse, 1.0, None, 0.1, br, 3, p, 1.0,
                                                 None, 0.1, be, 3, p, None)
    rc = lib.tq_se_gate_f32(*args(4, 0, 8))
    assert rc == 1 and b"bad shape" in lib.tq_last_error()
    rc = lib.tq_se_gate_f32(*args(4, 96, 8, xp=None))
    assert rc == 1 and b"null" in lib.tq_last_error()
    rc = lib.tq_se_gate_f32(*args(4, 96, 8, br=15))
    assert rc == 2 and b"<= 14" in lib.tq_last_error()
    rc = lib.tq_se_gate_f32(*args(4, 20000, 8))
    assert rc == 2 and b"LDS" in lib.tq_last_error()
    assert lib.tq_se_gate_f32(*args(0, 96, 8)) == 0
