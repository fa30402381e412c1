"""Functional TQ ops on torch tensors, all backed by libtq_hip.so (tq_native).

  tr(input, sf, bitwidth, group_size, num_keep_terms)     reference tr_cuda.tr, same contract
  tr_elementwise(x, sf, bitwidth, num_keep_terms)          group_size-1 TR of any dense layout
  tr_encode(w, sf, bitwidth, group_size, num_keep_terms)   TR(w) plus its integer term sums
  conv_engine(data_bits, weight_bits)                      "mfma" (fp16 codes) or "valu" (int16)
  pack_conv_weight(codes, engine)                          [O,I,KH,KW] int32 -> [O_pad, Kp] codes
  mfma_flush_steps(packed, data_bits)                      exactness window of the MFMA engine
  tr_conv2d(x, ...)                                        conv2d(TR(x), TR(w)) by term pairs

Two engines accumulate the same exact integer term-pair sums: the VALU engine (int16 codes,
v_dot2c_i32_i16) and the MFMA engine (fp16 codes, v_mfma_f32_32x32x16_f16 with exact fp32
windows flushed into int32, csrc/tr_conv_mfma.hip).  Their outputs are bit-identical; a
layer uses MFMA when its codes fit fp16 exactly (bitwidths <= 11) unless TQ_CONV_ENGINE=valu.

The TR ops (tr, tr_elementwise, tr_encode) take CUDA tensors (libtq_hip.so) and, as the
deliberate extension of SURVEY.md 8(b), CPU tensors (libtq_host.so, the OpenMP host TR op --
bit-identical results; the reference rejects CPU tensors and so cannot run its own MNIST CPU
config).  The term-pair conv/linear ops are GPU-only.
Errors mirror the reference boundary (kernels/tr_cuda.cpp:12-18): RuntimeError for a tensor on
any other device or a non-contiguous input, a RuntimeError for an unsupported dtype,
IndexError for < 2 dims.
"""
import numpy as np
import torch

import tq_native

import os

ACT_CHANNEL_ALIGN = 8   # 16-bit codes per 16-byte vector
K_ALIGN = 32            # codes per K-step of the VALU term-pair kernel
K_ALIGN_MFMA = 64       # codes per K-step of the MFMA term-pair kernel
MAX_CODE_BITS = 14      # |code| <= 2^bitwidth must fit int16
MAX_F16_CODE_BITS = 11  # |code| <= 2048: every integer is an fp16 value
FP32_EXACT = 2**24      # integers up to here are exact fp32 values

_kernel_hook = None


def set_kernel_hook(hook):
    """Install ``hook(name, work, launch_fn, nbytes)`` around the term-pair path's kernel
    launches (bench.py times them with HIP events on the launch stream; ``nbytes`` = the
    launch's algorithmic HBM bytes where the caller states them, else 0); None removes it."""
    global _kernel_hook
    _kernel_hook = hook


def _launch(name, work, fn, nbytes=0):
    return fn() if _kernel_hook is None else _kernel_hook(name, work, fn, nbytes)


def _check_input(input):
    # kernels/tr_cuda.cpp:12-18 (CHECK_CUDA, CHECK_CONTIGUOUS) and the dispatch dtype check
    if not isinstance(input, torch.Tensor):
        raise TypeError("tr(): input must be a torch.Tensor")
    if input.device.type not in ("cuda", "cpu"):
        raise RuntimeError("input must be a CUDA (or CPU) tensor")
    if not input.is_contiguous():
        raise RuntimeError("input must be contiguous")
    if input.dtype not in (torch.float32, torch.float64):
        raise RuntimeError('"tr_cuda" not implemented for \'%s\'' % str(input.dtype).replace(
            "torch.", "").capitalize())
    if input.dim() < 2:
        # input.size(1) on a 0-/1-D tensor (kernels/tr_cuda_kernel.cu:135)
        raise IndexError("Dimension out of range (expected to be in range of [-%d, %d], but "
                         "got 1)" % (max(input.dim(), 1), max(input.dim() - 1, 0)))


def tr(input, sf, bitwidth, group_size, num_keep_terms):
    """Term-revealing op: ``tr_cuda.tr`` of the reference (kernels/tr_cuda.cpp:20-28).

    Returns a new tensor of the input's shape and dtype holding sf * (sum of the kept HESE
    terms) per element; ``sf`` is narrowed to float32 as at the pybind boundary."""
    _check_input(input)
    out = torch.empty_like(input, memory_format=torch.contiguous_format)
    if input.numel() == 0:
        return out
    run = tq_native.tr_into if input.is_cuda else tq_native.tr_into_host
    return run(input, out, float(sf), int(bitwidth), int(group_size), int(num_keep_terms))


def tr_elementwise(x, sf, bitwidth, num_keep_terms):
    """group_size-1 TR (the activation call, tr_layer.py:96-99) on any dense tensor.

    Elementwise, so a channels_last (or otherwise permuted but dense) tensor is processed in
    its own memory order and the result keeps the input's strides."""
    if x.device.type not in ("cuda", "cpu"):
        raise RuntimeError("input must be a CUDA (or CPU) tensor")
    if x.dtype not in (torch.float32, torch.float64):
        raise RuntimeError('"tr_cuda" not implemented for \'%s\'' % str(x.dtype))
    if x.is_contiguous():
        flat = x.view(1, -1, 1, 1)
        return tr(flat, sf, bitwidth, 1, num_keep_terms).view(x.shape)
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        base = x.permute(0, 2, 3, 1)  # contiguous NHWC view of the same storage
        out = tr(base.reshape(1, -1, 1, 1), sf, bitwidth, 1, num_keep_terms)
        return out.view(base.shape).permute(0, 3, 1, 2)
    return tr(x.contiguous().view(1, -1, 1, 1), sf, bitwidth, 1,
              num_keep_terms).view(x.shape)


def histc_track(x, hist, minv, maxv, counts):
    """``hist += torch.histc(x, hist.numel(), minv, maxv)`` (tr_layer.py:91-94) for an fp32
    CUDA tensor on the tracking-histogram kernel (exact integer counts, tq_histc_f32); the
    memory order of x does not matter.  ``counts``: zeroed int64 scratch [nbins] on x's device.
    Other tensors (CPU, float64) take torch.histc itself, as the reference does."""
    if not x.is_cuda or x.dtype != torch.float32:
        hist += torch.histc(x, hist.numel(), minv, maxv)
        return hist
    dense = x.is_contiguous() or (x.dim() == 4 and
                                  x.is_contiguous(memory_format=torch.channels_last))
    if not dense:
        x = x.contiguous()
    if x.data_ptr() % 16:
        x = x.clone()
    return tq_native.histc_accumulate(x, hist, minv, maxv, counts)


def tr_encode(w, sf, bitwidth, group_size, num_keep_terms):
    """(TR(w), v) with TR(w) == v * fp32(sf) exactly; v int32 with w's shape."""
    _check_input(w)
    if w.dtype != torch.float32:
        raise RuntimeError("tr_encode: float32 only")
    out = torch.empty_like(w)
    codes = torch.empty(w.shape, dtype=torch.int32, device=w.device)
    if w.numel() == 0:
        return out, codes
    run = tq_native.tr_into if w.is_cuda else tq_native.tr_into_host
    run(w, out, float(sf), int(bitwidth), int(group_size), int(num_keep_terms), codes=codes)
    return out, codes


def round_up(v, m):
    return (v + m - 1) // m * m


def act_channels(c):
    return round_up(c, ACT_CHANNEL_ALIGN)


def conv_engine(data_bits, weight_bits):
    """Term-pair engine for a layer: "mfma" when activation and weight codes are exact fp16
    values (both bitwidths <= 11), else "valu".  TQ_CONV_ENGINE=valu forces the VALU engine
    (the two are bit-identical; tests compare them)."""
    forced = os.environ.get("TQ_CONV_ENGINE", "").lower()
    if forced not in ("", "mfma", "valu"):
        raise RuntimeError("TQ_CONV_ENGINE must be 'mfma' or 'valu' (got %r)" % forced)
    if forced == "valu":
        return "valu"
    if max(int(data_bits), int(weight_bits)) <= MAX_F16_CODE_BITS:
        return "mfma"
    return "valu"


def code_dtype(engine):
    return torch.float16 if engine == "mfma" else torch.int16


def pack_conv_weight(codes, engine="valu"):
    """[O, I, KH, KW] int32 term sums -> [O_pad, Kp] codes with k = (kh*KW + kw)*Cp + c:
    int16 with Kp % 32 == 0 (VALU engine) or float16 with Kp % 64 == 0 (MFMA engine).

    Layout plumbing done once per layer at construction; returns (packed, Cp)."""
    o, i, kh, kw = codes.shape
    cp = act_channels(i)
    t = codes.permute(0, 2, 3, 1)  # O, KH, KW, I
    if cp != i:
        t = torch.nn.functional.pad(t, (0, cp - i))
    t = t.reshape(o, kh * kw * cp)
    kp = round_up(kh * kw * cp, K_ALIGN_MFMA if engine == "mfma" else K_ALIGN)
    o_pad = round_up(o, tq_native.conv2d_cout_align())
    dtype = code_dtype(engine)
    if engine == "mfma" and codes.numel() and codes.abs().max().item() > 2**MAX_F16_CODE_BITS:
        raise RuntimeError("pack_conv_weight: codes exceed the exact fp16 range")
    packed = torch.zeros((o_pad, kp), dtype=dtype, device=codes.device)
    packed[:o, :kh * kw * cp] = t.to(dtype)
    return packed.contiguous(), cp


def _window_sums(steps, nonneg):
    """Per-window magnitude bounds from per-K-step code sums v [..., S, 64]: sum|v| in
    general; max(sum of positive v, sum of |negative v|) when the activation codes are known
    to be non-negative (post-ReLU): every partial sum of v_x * v_w with 0 <= v_x <= 2^db then
    lies in [-2^db * N, 2^db * P], in any association order."""
    if nonneg:
        return [steps.clamp(min=0).sum(-1), (-steps).clamp(min=0).sum(-1)]
    return [steps.abs().sum(-1)]


def _longest_window(parts, lim, dim):
    """Largest n such that every window of n consecutive steps along ``dim`` of every part
    sums to at most lim (0 if none)."""
    s = parts[0].shape[dim]
    cs = [torch.nn.functional.pad(p.cumsum(dim), (1, 0)) for p in parts]
    best = 0
    for n in range(1, s + 1):
        if max((c.narrow(dim, n, s + 1 - n) - c.narrow(dim, 0, s + 1 - n)).max().item()
               for c in cs) > lim:
            break
        best = n
    return best, s


def mfma_flush_steps(packed, data_bits, nonneg=False):
    """Exactness window of the MFMA engine for fp16 weight codes ``packed`` [O_pad, Kp]
    against activation codes of ``data_bits`` bits (|v_x| <= 2^data_bits).

    Returns the largest n such that every window of n consecutive K-steps (64 codes) of every
    row satisfies 2^data_bits * sum|v_w| <= 2^24 -- then every fp32 partial sum inside the
    window is an exact integer -- as the kernel's flush interval: 0 if the whole K range
    qualifies (no flush needed), -1 if not even one K-step does (the layer must use the VALU
    engine).  ``nonneg``: the bound for non-negative activation codes (_window_sums)."""
    o_pad, kp = packed.shape
    steps = packed.double().view(o_pad, kp // K_ALIGN_MFMA, K_ALIGN_MFMA)
    lim = float(FP32_EXACT) / float(2**int(data_bits))
    best, s = _longest_window(_window_sums(steps, nonneg), lim, 1)
    if best == 0:
        return -1
    return 0 if best == s else best


STEM_W_EXP = 10      # csrc/tq_stem_conv.hip kStemWExp: weights are packed as w * 2^10
STEM_W_MAX = 32.0    # |w| * 2^10 stays below the fp16 range (65504)


def pack_stem_weight(w):
    """ResNet stem conv weight [64, 3, 7, 7] fp32 -> [2, 64, 192] fp16 bits (int16 tensor) for
    tq_stem_conv_pool_encode: the 7x7 kernel padded to 8x8 with a leading zero tap, in
    space-to-depth K order (sy, sx, sub_r, sub_c, c), scaled by 2^10 (exact) and split into
    two fp16 parts w * 2^10 = w0 + w1 + e (w0 = RN16, w1 = RN16 of the exact remainder,
    |e| <= 2^-22 |w| * 2^10 while w1 is normal).  Raises RuntimeError for weights the fp16
    range cannot hold (|w| > 32 or non-finite); the executor then keeps the unfused stem."""
    if tuple(w.shape) != (64, 3, 7, 7) or w.dtype != torch.float32:
        raise RuntimeError("pack_stem_weight: expects a [64, 3, 7, 7] float32 weight")
    wd = w.detach()
    if not bool(torch.isfinite(wd).all()) or float(wd.abs().max()) > STEM_W_MAX:
        raise RuntimeError("pack_stem_weight: weights must be finite with |w| <= %g"
                           % STEM_W_MAX)
    w8 = torch.zeros((64, 3, 8, 8), dtype=torch.float32, device=w.device)
    w8[:, :, 1:, 1:] = wd * (2.0 ** STEM_W_EXP)
    # [o, c, sy, sub_r, sx, sub_c] -> [o, sy, sx, sub_r, sub_c, c]
    k = w8.view(64, 3, 4, 2, 4, 2).permute(0, 2, 4, 3, 5, 1).reshape(64, 192)
    w0 = k.to(torch.float16)
    w1 = (k - w0.float()).to(torch.float16)
    return torch.stack([w0, w1]).contiguous().view(torch.int16)


# Relative error of the fused stem's split conv per unit of |x|_2 |w|_2 (the conv position's
# input window norm times the output channel's weight norm; Cauchy-Schwarz bounds the
# magnitude sum S = sum |x| |w| by it):
#  * the split: x w - (x0 w0 + x0 w1 + x1 w0) = x1 w1 + x ew + x1 ew + ex w with |x1| <=
#    2^-11 |x|, |ex|, |ew| <= 2^-22 |.|: <= 3 * 2^-22 S = 6 * 2^-23 S;
#  * the accumulation: v_mfma_f32_16x16x32_f16 sums each 8-product group aligned to its
#    largest product and truncated below that product's 24-bit window, adds the groups and C
#    wider, and rounds once without a sticky bit (tools/probes/mfma_align.hip,
#    profiles/r06_mfma_rounding.txt): per MFMA within 2^-23 (7 sum |ab| + |D|).  18 MFMAs
#    accumulate into one output and every |D| <= S (1 + 2^-10): <= 25 * 2^-23 S.
# Together <= 31 * 2^-23; 34 * 2^-23 leaves a 10 % margin (the kernel adds 2^-8 for the
# norms' own rounding).  Measured per-MFMA errors stay below 4.7 * 2^-24 (|C| + sum |ab|) on
# 10^6 random outputs (tools/probes/mfma_rounding.hip).
STEM_ERR_REL = 34.0 * 2.0 ** -23


def pack_stem_exact(w):
    """ResNet stem conv weight [64, 3, 7, 7] fp32 -> (w64, wbound) for the fused stem's exact
    fix-up (tq_stem_conv_pool_encode): w64 the weights in fp64 as [64, 7, 7, 3] (kernel row,
    column, input channel), wbound[c] an fp32 upper bound of STEM_ERR_REL * |w[c]|_2 (plus
    2^-13 of slack for the fp16 splits' subnormal weight remainders, 2^-35 |x| each)."""
    if tuple(w.shape) != (64, 3, 7, 7) or w.dtype != torch.float32:
        raise RuntimeError("pack_stem_exact: expects a [64, 3, 7, 7] float32 weight")
    wd = w.detach()
    w64 = wd.double().permute(0, 2, 3, 1).contiguous()
    l2 = wd.double().pow(2).sum(dim=(1, 2, 3)).sqrt().cpu().numpy()
    b = (STEM_ERR_REL * (l2 * (1.0 + 2.0 ** -10) + 2.0 ** -13)).astype(np.float32)
    b = np.nextafter(b, np.float32(np.inf))  # rounded up
    return w64, torch.from_numpy(b).to(w.device)


def mfma_flush_chunk(packed, data_bits, cp, ntaps, nonneg=False):
    """mfma_flush_steps for kernels that walk K chunk-major (tq.h ``kc_chunk``): the largest
    n such that every window of n consecutive filter taps of one 64-code channel chunk
    satisfies 2^data_bits * sum|v_w| <= 2^24 in every row; 0 if a whole chunk qualifies
    (the kernel also flushes at every chunk end), -1 if not even one step does or if Cp is
    not a multiple of 64 (no chunk-major kernel runs then; -1 lets the library derive a
    conservative value from kc_steps).  ``nonneg`` as in mfma_flush_steps."""
    if cp % K_ALIGN_MFMA:
        return -1
    o_pad, kp = packed.shape
    nch = cp // K_ALIGN_MFMA
    steps = packed.double().view(o_pad, kp // K_ALIGN_MFMA, K_ALIGN_MFMA)
    steps = steps[:, :ntaps * nch].reshape(o_pad, ntaps, nch, K_ALIGN_MFMA).permute(0, 2, 1, 3)
    lim = float(FP32_EXACT) / float(2**int(data_bits))
    best, _ = _longest_window(_window_sums(steps, nonneg), lim, 2)  # [O, c, tap] windows
    if best == 0:
        return -1
    return 0 if best == ntaps else best


def conv_out_size(h, k, s, p, d):
    return (h + 2 * p - d * (k - 1) - 1) // s + 1


def tr_conv2d(x, sf_x, data_bits, data_terms, w_packed, cp, sf_w, bias, out_channels,
              kernel_size, stride, padding, dilation, kc_steps=0, kc_chunk=-1):
    """conv2d(TR(x), TR(w)) + bias by exact term-pair accumulation (groups = 1).

    x: fp32 [N, C, H, W] CUDA tensor, NCHW-contiguous or channels_last.  The output has the
    conv's shape and the input's memory format (as cuDNN/MIOpen convs do).  The engine
    follows ``w_packed``'s dtype (pack_conv_weight): float16 -> MFMA with flush interval
    ``kc_steps`` (mfma_flush_steps), int16 -> VALU."""
    if not x.is_cuda:
        raise RuntimeError("input must be a CUDA tensor")
    if x.dtype != torch.float32 or x.dim() != 4:
        raise RuntimeError("tr_conv2d: expects a 4-D float32 input")
    n, c, h, w = x.shape
    if act_channels(c) != cp:
        raise RuntimeError("tr_conv2d: input has %d channels, weights expect %d" % (c, cp))
    nhwc = (not x.is_contiguous()) and x.is_contiguous(memory_format=torch.channels_last)
    if not nhwc and not x.is_contiguous():
        x = x.contiguous()
    kh, kw = kernel_size
    ho = conv_out_size(h, kh, stride[0], padding[0], dilation[0])
    wo = conv_out_size(w, kw, stride[1], padding[1], dilation[1])
    codes = torch.empty((n, h, w, cp), dtype=w_packed.dtype, device=x.device)
    _launch("act_encode", 4 * n * c * h * w + 2 * n * h * w * cp,
            lambda: tq_native.act_encode(x, nhwc, float(sf_x), int(data_bits), int(data_terms),
                                         codes))
    fmt = torch.channels_last if nhwc else torch.contiguous_format
    out = torch.empty((n, out_channels, ho, wo), dtype=torch.float32, device=x.device,
                      memory_format=fmt)
    # one rounding of the exact integer sum: scale = fp32(sf_x) * fp32(sf_w) in double
    scale = float(np.float32(sf_x)) * float(np.float32(sf_w))
    if bias is not None:
        bias = bias.detach().to(torch.float32).contiguous()
    _launch("conv2d_termpair", n * ho * wo * out_channels * c * kh * kw,
            lambda: tq_native.conv2d_termpair(codes, w_packed, out_channels, kh, kw, stride,
                                              padding, dilation, scale, bias, out, nhwc,
                                              kc_steps, kc_chunk))
    return out


def static_padding(conv):
    """(top, bottom, left, right) zero padding a Conv2dStaticSamePadding-style module applies
    before its convolution (efficientnet_pytorch semantics), else zeros."""
    pad = getattr(conv, "static_padding", None)
    if pad is None or not isinstance(pad, torch.nn.ZeroPad2d):
        return (0, 0, 0, 0)
    left, right, top, bottom = pad.padding
    return (top, bottom, left, right)


def pack_dw_weight(codes):
    """[C, 1, KH, KW] int32 term sums -> int32 [KH*KW, Cp] (tap-major, channel fastest)."""
    c, _, kh, kw = codes.shape
    cp = act_channels(c)
    packed = torch.zeros((kh * kw, cp), dtype=torch.int32, device=codes.device)
    packed[:, :c] = codes.reshape(c, kh * kw).t()
    return packed.contiguous(), cp


def tr_dwconv2d(x, sf_x, data_bits, data_terms, w_packed, cp, sf_w, bias, channels,
                kernel_size, stride, padding, dilation, pad_tblr=(0, 0, 0, 0)):
    """Depthwise conv2d(TR(x), TR(w)) + bias by exact term-pair accumulation."""
    if not x.is_cuda:
        raise RuntimeError("input must be a CUDA tensor")
    if x.dtype != torch.float32 or x.dim() != 4:
        raise RuntimeError("tr_dwconv2d: expects a 4-D float32 input")
    n, c, h, w = x.shape
    if c != channels:
        raise RuntimeError("tr_dwconv2d: input has %d channels, weights expect %d" % (c,
                                                                                  channels))
    nhwc = (not x.is_contiguous()) and x.is_contiguous(memory_format=torch.channels_last)
    if not nhwc and not x.is_contiguous():
        x = x.contiguous()
    kh, kw = kernel_size
    top, bottom, left, right = pad_tblr
    ho = conv_out_size(h + top + bottom, kh, stride[0], padding[0], dilation[0])
    wo = conv_out_size(w + left + right, kw, stride[1], padding[1], dilation[1])
    codes = torch.empty((n, h, w, cp), dtype=torch.int16, device=x.device)
    _launch("act_encode", 4 * n * c * h * w + 2 * n * h * w * cp,
            lambda: tq_native.act_encode(x, nhwc, float(sf_x), int(data_bits), int(data_terms),
                                         codes))
    fmt = torch.channels_last if nhwc else torch.contiguous_format
    out = torch.empty((n, c, ho, wo), dtype=torch.float32, device=x.device, memory_format=fmt)
    scale = float(np.float32(sf_x)) * float(np.float32(sf_w))
    if bias is not None:
        bias = bias.detach().to(torch.float32).contiguous()
    _launch("dwconv2d_termpair", n * ho * wo * c * kh * kw,
            lambda: tq_native.dwconv2d_termpair(codes, c, w_packed, kh, kw, stride,
                                                (top + padding[0], left + padding[1]),
                                                dilation, scale, bias, out, nhwc),
            2 * codes.numel() + 4 * out.numel() + 4 * w_packed.numel())
    return out


MAX_WIDE_WEIGHT_BITS = 16  # tq_conv2d_termpair_wide: |v_x| <= 2^14, |v_w| <= 2^16


def pack_wide_weight(codes):
    """[O, I, KH, KW] int32 term sums -> int32 [O, KH*KW*Cp] with k = (kh*KW + kw)*Cp + c
    (tq_conv2d_termpair_wide); returns (packed, Cp)."""
    o, i, kh, kw = codes.shape
    cp = act_channels(i)
    t = codes.permute(0, 2, 3, 1)
    if cp != i:
        t = torch.nn.functional.pad(t, (0, cp - i))
    return t.reshape(o, kh * kw * cp).to(torch.int32).contiguous(), cp


def tr_conv2d_wide(x, sf_x, data_bits, data_terms, w_packed, cp, sf_w, bias, out_channels,
                   kernel_size, stride, padding, dilation):
    """conv2d(TR(x), TR(w)) + bias by exact term-pair accumulation with int32 weight codes
    (weight bit widths 15-16: EfficientNet-b0's squeeze-excite convs), int64 sums."""
    if not x.is_cuda:
        raise RuntimeError("input must be a CUDA tensor")
    if x.dtype != torch.float32 or x.dim() != 4:
        raise RuntimeError("tr_conv2d_wide: expects a 4-D float32 input")
    n, c, h, w = x.shape
    if act_channels(c) != cp:
        raise RuntimeError("tr_conv2d_wide: input has %d channels, weights expect %d" % (c, cp))
    nhwc = (not x.is_contiguous()) and x.is_contiguous(memory_format=torch.channels_last)
    if not nhwc and not x.is_contiguous():
        x = x.contiguous()
    kh, kw = kernel_size
    ho = conv_out_size(h, kh, stride[0], padding[0], dilation[0])
    wo = conv_out_size(w, kw, stride[1], padding[1], dilation[1])
    codes = torch.empty((n, h, w, cp), dtype=torch.int16, device=x.device)
    _launch("act_encode", 4 * n * c * h * w + 2 * n * h * w * cp,
            lambda: tq_native.act_encode(x, nhwc, float(sf_x), int(data_bits), int(data_terms),
                                         codes))
    fmt = torch.channels_last if nhwc else torch.contiguous_format
    out = torch.empty((n, out_channels, ho, wo), dtype=torch.float32, device=x.device,
                      memory_format=fmt)
    scale = float(np.float32(sf_x)) * float(np.float32(sf_w))
    if bias is not None:
        bias = bias.detach().to(torch.float32).contiguous()
    _launch("conv2d_termpair_wide", n * ho * wo * out_channels * c * kh * kw,
            lambda: tq_native.conv2d_termpair_wide(codes, w_packed, out_channels, kh, kw, stride,
                                                   padding, dilation, scale, bias, out, nhwc))
    return out


def tr_linear(x, sf_x, data_bits, data_terms, w_packed, cp, sf_w, bias, out_features,
              kc_steps=0, kc_chunk=-1):
    """linear(TR(x), TR(w)) + bias by exact term-pair accumulation: the rows of x are the
    pixels of a 1x1 term-pair conv (channels_last [M, C, 1, 1] is x's own memory)."""
    shape = x.shape
    x2 = x.reshape(-1, shape[-1]).contiguous()
    m = x2.shape[0]
    xc = x2.view(m, 1, 1, shape[-1]).permute(0, 3, 1, 2)  # channels_last view, no copy
    y = tr_conv2d(xc, sf_x, data_bits, data_terms, w_packed, cp, sf_w, bias, out_features,
                  (1, 1), (1, 1), (0, 0), (1, 1), kc_steps, kc_chunk)
    return y.permute(0, 2, 3, 1).reshape(*shape[:-1], out_features)
