"""Term-quantization module API -- the drop-in for the reference's tr_layer.py.

Same public names, constructor signatures, attributes and behaviour as the reference
(tr_layer.py:1-201): ``tr_cuda`` (an object with ``.tr``), ``hese``, ``mse_profile``,
``compute_compressed_hese``, ``set_tr_tracking``, ``LinearQuantize``, ``TRConv2dLayer``,
``TRLinearLayer`` and ``TRLSTMLayer``.  Underneath, every TR runs in the MI355X HIP library
(libtq_hip.so), and a converted Conv2d no longer runs a dense fp32 conv of fake-quantized
tensors: it accumulates term pairs exactly in the term-pair kernel (tq_ops.tr_conv2d).
"""
import math
import os

import numpy as np
import torch
import torch.nn as nn

import tq_native
import tq_ops


class _TRExtension(object):
    """Stands where ``tr_cuda = load('tr_cuda', [...])`` stood (tr_layer.py:7): a module-like
    object whose ``tr`` is the reference pybind entry (kernels/tr_cuda.cpp:20-28)."""

    __name__ = "tr_cuda"

    @staticmethod
    def tr(input, sf, bitwidth, group_size, num_keep_terms):
        return tq_ops.tr(input, sf, bitwidth, group_size, num_keep_terms)


tr_cuda = _TRExtension()


def hese(number):
    """tr_layer.hese (tr_layer.py:9-41): the run-based HESE variant used for parameter-bit
    counting.  Each run of ones from bit a up to bit b becomes (-2^a, +2^(b+1)), and a run of
    length one collapses to the single term +2^a ("merging neighbors hack").  Terms come out
    least significant run first, signed by the number's sign."""
    sign = -1 if number < 0 else 1
    q = abs(int(number))
    terms = []
    i = 0
    while q >> i:
        if (q >> i) & 1:
            j = i
            while (q >> j) & 1:
                j += 1
            if j == i + 1:
                terms.append(sign * (1 << i))
            else:
                terms.append(-sign * (1 << i))
                terms.append(sign * (1 << j))
            i = j
        else:
            i += 1
    return terms


def _hese_len_tensor(q):
    """len(hese(q)) for every element of an integer tensor: 2 terms per run of ones, 1 for
    a run of length one."""
    q = q.abs().to(torch.int64)
    starts = q & ~(q << 1)
    singles = starts & ~(q >> 1)

    def popcount(v):
        c = torch.zeros_like(v)
        while bool((v != 0).any()):
            c += v & 1
            v = v >> 1
        return c

    return 2 * popcount(starts) - popcount(singles)


def mse_profile(hist, minv, maxv, bit_width, terms):
    """Activation scale factor by weighted-MSE search (tr_layer.py:43-54).

    Same candidate grid (2048 fp32 sfs in linspace(1e-8, maxv)) and the same histogram grid
    as the reference; all 2048 candidates are scored in one HIP launch (tq_mse_profile) and
    the first arg-min is returned as a Python float, like ``sfs[min_idx]``."""
    device = hist.device
    x = torch.linspace(minv, maxv, len(hist)).to(device)
    sfs_list = torch.linspace(1e-8, maxv, 2048).tolist()
    sfs = torch.tensor(sfs_list, dtype=torch.float32, device=device)
    h = hist.detach().to(device=device, dtype=torch.float32).contiguous()
    # the HIP kernel for a GPU histogram, the host library (same errs) for a CPU one
    run = tq_native.mse_profile if hist.is_cuda else tq_native.mse_profile_host
    errs = run(x.contiguous(), h, sfs, bit_width, terms)
    min_idx = int(torch.argmin(errs).item())
    return sfs_list[min_idx]


def compute_compressed_hese(w, sf, weight_terms):
    """Parameter bits of HESE-compressed weights (tr_layer.py:57-63).  The reference loops
    over every weight in Python; this counts the same terms with tensor ops."""
    exp_bits = math.ceil(math.log2(weight_terms))
    bit_width = exp_bits + 2  # 1 for sign, 1 for barrier
    w = (w / sf).int()
    return int(bit_width * int(_hese_len_tensor(w).sum().item()))


def set_tr_tracking(model, tracking):
    """Switch every TR layer between calibration and quantized mode (tr_layer.py:66-76)."""
    for name, layer in model.named_modules():
        if isinstance(layer, (TRLinearLayer, TRLSTMLayer, TRConv2dLayer)):
            module_keys = name.split('.')
            module = model
            for k in module_keys[:-1]:
                module = module._modules[k]

            module._modules[module_keys[-1]].tracking(tracking)

    return model


class LinearQuantize(nn.Module):
    """Per-layer activation quantizer (tr_layer.py:78-104).

    While ``tracking``: accumulates an 8192-bin histogram over [-50, 50] and returns x.
    Afterwards: TR with group size 1, ``data_bits`` bits and ``data_terms`` kept terms."""

    def __init__(self, data_bits, data_terms):
        super(LinearQuantize, self).__init__()
        self.sf = 1
        self.num_bins = 8192
        self.minv = -50
        self.maxv = 50
        self.register_buffer('hist_bins', torch.Tensor(self.num_bins).zero_())
        self.tracking = True
        self.data_bits = data_bits
        self.data_terms = data_terms

    def forward(self, x):
        if self.tracking:
            # the tracking-histogram kernel for GPU tensors: exact counts (torch.histc's fp32
            # atomic counts stop at 2^24 per bin), the same bins otherwise
            if x.is_cuda and self.hist_bins.is_cuda and self.hist_bins.is_contiguous():
                counts = self.__dict__.get('_hist_counts')
                if counts is None or counts.device != x.device or \
                        counts.numel() != self.num_bins:
                    counts = torch.zeros(self.num_bins, dtype=torch.int64, device=x.device)
                    self.__dict__['_hist_counts'] = counts
                tq_ops.histc_track(x, self.hist_bins, self.minv, self.maxv, counts)
            else:
                self.hist_bins += torch.histc(x, self.num_bins, self.minv, self.maxv)
            return x

        return tq_ops.tr_elementwise(x, self.sf, self.data_bits, self.data_terms)

    def finish_tracking(self):
        self.sf = mse_profile(self.hist_bins, self.minv, self.maxv,
                              self.data_bits, self.data_terms)
        self.tracking = False


def _kc_chunk(packed, engine, data_bits, cp, ntaps):
    """Exactness window for the chunk-major MFMA engine (tq_ops.mfma_flush_chunk)."""
    if engine != "mfma":
        return 0
    return tq_ops.mfma_flush_chunk(packed, data_bits, cp, ntaps)


def _pack_termpair(codes, data_bits, weight_bits):
    """Pack int32 weight term sums [O, I, KH, KW] for the layer's term-pair engine:
    (packed, Cp, engine, kc_steps).  MFMA when the codes are exact fp16 values and one K-step
    of products stays inside fp32's exact-integer range, else VALU (int16)."""
    engine = tq_ops.conv_engine(data_bits, weight_bits)
    if engine == "mfma":
        packed, cp = tq_ops.pack_conv_weight(codes, "mfma")
        kc = tq_ops.mfma_flush_steps(packed, data_bits)
        if kc >= 0:
            return packed, cp, "mfma", kc
    packed, cp = tq_ops.pack_conv_weight(codes, "valu")
    return packed, cp, "valu", 0


def _w_sf(w, weight_bits):
    max_wq = 2**(weight_bits - 1)
    return w.abs().max().item() / max_wq


class TRConv2dLayer(nn.Module):
    """Conv2d with term-revealed weights and activations (tr_layer.py:106-132).

    Construction TRs the weight with group size ``group_size`` and budget ``num_terms`` and
    keeps the fake-quantized tensor as ``self.conv.weight`` (so ``profile_model`` and any
    caller reading the weight see the reference values).  It also keeps the integer term
    sums, packed for the term-pair kernels, in the ``w_codes`` buffer.

    forward: while tracking, ``self.conv`` on the unquantized input (the reference returns x
    from the quantizer while tracking); afterwards conv2d(TR(x), TR(w)) + bias by exact
    term-pair accumulation -- ``self.mode``:
      "termpair"   groups == 1, data/weight bits <= 14: tq_ops.tr_conv2d on the MFMA engine
                   (fp16 codes, bits <= 11; ``self.engine`` "mfma") or the VALU engine
                   (int16 codes, ``self.engine`` "valu") -- bit-identical results
      "depthwise"  groups == C_in == C_out, weight bits <= 22: tq_ops.tr_dwconv2d
      "wide"       groups == 1, weight bits 15-16 (the (16, 1, 16) squeeze-excite convs of
                   EfficientNet-b0): tq_ops.tr_conv2d_wide, int32 weight codes, int64 sums
      "reference"  anything else: the reference composition self.conv(self.input_quant(x))
                   with the HIP TR op (``self.termpair`` is True only for "termpair").
    The term-pair kernels are GPU kernels: a CPU input (the MNIST CPU config)
    runs the reference composition with the host TR op (libtq_host.so) and torch's CPU conv
    on the same TR'd weights.  A CUDA input never takes that path."""

    def __init__(self, conv_layer, data_bits=8, data_terms=4, weight_bits=8,
                 group_size=1, num_terms=8):
        super(TRConv2dLayer, self).__init__()
        device = conv_layer.weight.device
        self.data_bits = data_bits
        self.data_terms = data_terms
        self.input_quant = LinearQuantize(data_bits, data_terms).to(device)
        self.group_size = group_size
        self.num_terms = num_terms
        self.weight_bits = weight_bits
        w = conv_layer.weight
        self.w_sf = _w_sf(w, weight_bits)
        c = conv_layer
        plain = (getattr(c, 'padding_mode', 'zeros') == 'zeros'
                 and not isinstance(c.padding, str) and w.dtype == torch.float32
                 and data_bits <= tq_ops.MAX_CODE_BITS)
        mode = "reference"
        if plain and c.groups == 1 and weight_bits <= tq_ops.MAX_CODE_BITS:
            mode = "termpair"
        elif (plain and c.groups > 1 and c.groups == c.in_channels == c.out_channels
              and weight_bits <= 22):
            mode = "depthwise"
        elif plain and c.groups == 1 and weight_bits <= tq_ops.MAX_WIDE_WEIGHT_BITS:
            mode = "wide"
        packed = None
        if mode == "wide":
            wq, codes = tq_ops.tr_encode(w.detach().contiguous(), self.w_sf, weight_bits,
                                         group_size, num_terms)
            packed, cp = tq_ops.pack_wide_weight(codes)
        elif mode != "reference":
            wq, codes = tq_ops.tr_encode(w.detach().contiguous(), self.w_sf, weight_bits,
                                         group_size, num_terms)
            # int32 accumulator bound: sum_k |v_w| * max|v_x| (|v_x| <= 2^data_bits)
            bound = codes.abs().to(torch.int64).flatten(1).sum(1).max().item() << data_bits
            if bound >= 2**31:
                mode = "reference"
            elif mode == "termpair":
                packed, cp, self.engine, self.kc_steps = _pack_termpair(codes, data_bits,
                                                                        weight_bits)
                ntaps = codes.shape[2] * codes.shape[3]
                self.kc_chunk = _kc_chunk(packed, self.engine, data_bits, cp, ntaps)
                # wider windows for callers whose activation codes are post-ReLU (>= 0): the
                # fused executor (tq_fuse.py); the module path keeps the general windows
                self.kc_steps_nonneg, self.kc_chunk_nonneg = self.kc_steps, self.kc_chunk
                if self.engine == "mfma":
                    self.kc_steps_nonneg = tq_ops.mfma_flush_steps(packed, data_bits, True)
                    self.kc_chunk_nonneg = tq_ops.mfma_flush_chunk(packed, data_bits, cp,
                                                                   ntaps, True)
            else:
                packed, cp = tq_ops.pack_dw_weight(codes)
        else:
            wq = tr_cuda.tr(w, self.w_sf, weight_bits, self.group_size, self.num_terms)
        self.mode = mode
        self.termpair = mode == "termpair"
        if not self.termpair:
            self.engine, self.kc_steps, self.kc_chunk = None, 0, 0
            self.kc_steps_nonneg, self.kc_chunk_nonneg = 0, 0
        self.register_buffer('w_codes', packed)
        if packed is not None:
            self.act_channels = cp
        conv_layer.weight = nn.Parameter(wq)
        self.conv = conv_layer

    def forward(self, x):
        if self.input_quant.tracking or self.mode == "reference" or not x.is_cuda:
            xq = self.input_quant(x)
            return self.conv(xq)
        c = self.conv
        pad = tq_ops.static_padding(c)
        if self.mode == "depthwise":
            return tq_ops.tr_dwconv2d(x, self.input_quant.sf, self.data_bits, self.data_terms,
                                      self.w_codes, self.act_channels, self.w_sf, c.bias,
                                      c.out_channels, c.kernel_size, c.stride, c.padding,
                                      c.dilation, pad)
        if any(pad):
            # TR(0) == 0: zero-padding before the encode equals padding the TR'd input
            x = torch.nn.functional.pad(x, (pad[2], pad[3], pad[0], pad[1]))
        if self.mode == "wide":
            return tq_ops.tr_conv2d_wide(x, self.input_quant.sf, self.data_bits,
                                         self.data_terms, self.w_codes, self.act_channels,
                                         self.w_sf, c.bias, c.out_channels, c.kernel_size,
                                         c.stride, c.padding, c.dilation)
        return tq_ops.tr_conv2d(x, self.input_quant.sf, self.data_bits, self.data_terms,
                                self.w_codes, self.act_channels, self.w_sf, c.bias,
                                c.out_channels, c.kernel_size, c.stride, c.padding, c.dilation,
                                self.kc_steps, self.kc_chunk)

    def tracking(self, tracking):
        if not tracking:
            self.input_quant.finish_tracking()
        else:
            self.input_quant.tracking = True


class TRLinearLayer(nn.Module):
    """Linear with term-revealed weights (tr_layer.py:134-160).

    Like the reference, forward returns ``self.linear(x)`` on the UNquantized input
    (tr_layer.py:152-154): only the weights are term-quantized.  The input quantizer still
    records its histogram while tracking; after calibration the reference computes TR(x) and
    discards it, which this layer skips (the output is identical).

    ``quantize_input=True`` (an addition, off by default) uses the quantized input as the
    reference evidently intended: linear(TR(x), TR(w)) by exact term-pair accumulation
    (the term-pair kernel as a 1x1 conv over the flattened rows)."""

    def __init__(self, linear_layer, data_bits=8, data_terms=4, weight_bits=8,
                 group_size=1, num_terms=8, quantize_input=False):
        super(TRLinearLayer, self).__init__()
        device = linear_layer.weight.device
        self.data_bits = data_bits
        self.data_terms = data_terms
        self.input_quant = LinearQuantize(data_bits, data_terms).to(device)
        self.group_size = group_size
        self.num_terms = num_terms
        self.weight_bits = weight_bits
        self.quantize_input = quantize_input
        w = linear_layer.weight
        self.w_sf = _w_sf(w, weight_bits)
        self.termpair = False
        self.engine, self.kc_steps, self.kc_chunk = None, 0, 0
        packed = None
        if (quantize_input and weight_bits <= tq_ops.MAX_CODE_BITS
                and data_bits <= tq_ops.MAX_CODE_BITS and w.dtype == torch.float32):
            wq, codes = tq_ops.tr_encode(w.detach().contiguous(), self.w_sf, weight_bits,
                                         group_size, num_terms)
            bound = codes.abs().to(torch.int64).sum(1).max().item() << data_bits
            if bound < 2**31:
                packed, self.act_channels, self.engine, self.kc_steps = _pack_termpair(
                    codes[:, :, None, None], data_bits, weight_bits)
                self.kc_chunk = _kc_chunk(packed, self.engine, data_bits, self.act_channels, 1)
                self.termpair = True
        else:
            wq = tr_cuda.tr(w, self.w_sf, weight_bits, self.group_size, self.num_terms)
        self.register_buffer('w_codes', packed)
        linear_layer.weight = nn.Parameter(wq)
        self.linear = linear_layer

    def forward(self, x):
        if self.input_quant.tracking:
            self.input_quant(x)
            return self.linear(x)
        if not self.quantize_input:
            return self.linear(x)
        if not self.termpair or not x.is_cuda:  # CPU input: host TR + torch's CPU linear
            return self.linear(self.input_quant(x))
        return tq_ops.tr_linear(x, self.input_quant.sf, self.data_bits, self.data_terms,
                                self.w_codes, self.act_channels, self.w_sf, self.linear.bias,
                                self.linear.out_features, self.kc_steps, self.kc_chunk)

    def tracking(self, tracking):
        if not tracking:
            self.input_quant.finish_tracking()
        else:
            self.input_quant.tracking = True


class TRLSTMLayer(nn.Module):
    """LSTM with term-revealed layer-0 weights and quantized inputs/hidden state
    (tr_layer.py:162-201); ``w_sf`` ends up as the weight_hh_l0 scale, as in the reference.

    The function is the reference's: ``self.lstm`` on TR(emb) and the TR'd (h0, c0) with
    the TR'd layer-0 weights (with ``termpair=False``, or for CPU inputs, that is literally
    the library LSTM, MIOpen on the GPU).

    ``termpair=True`` (the default for CUDA inputs) computes the same function with layer 0
    on the term-pair kernels: its input projection over all time steps is one exact
    term-pair GEMM, TR(emb) TR(W_ih)^T + b_ih (both operands term-revealed).  The recurrences
    then run as fused HIP step kernels launched from C++: for a 2-layer LSTM (LSTM-650) both
    layers in wavefront order from ONE ``tq_lstm_seq2_f32`` call (T + 1 launches of
    ``lstm_step2_kernel``: launch s runs layer 0's step s and layer 1's step s - 1, layer 1
    computing x_t W_ih^T inside its step); ``TQ_LSTM_WAVE=0`` runs one ``tq_lstm_seq_f32`` call
    per layer (T launches each), ``TQ_LSTM_SEQ=0`` the per-step hipBLASLt GEMM + one
    ``tq_lstm_cell_f32`` launch per step.  Layers >= 1 keep the reference's untouched weights
    and their quantized initial state.  fp32 results equal the reference composition to
    rounding, per log-prob (tests/test_gpu_lstm.py); the LSTM-650 chunk runs at 459-481 k
    tokens/s on the wavefront path vs 164-179 k for MIOpen's LSTM (bench d4)."""

    def __init__(self, lstm_layer, data_bits=8, data_terms=4, weight_bits=8,
                 group_size=1, num_terms=8, termpair=True):
        super(TRLSTMLayer, self).__init__()
        device = lstm_layer.weight_ih_l0.device
        self.data_bits = data_bits
        self.data_terms = data_terms
        self.input_quant = LinearQuantize(data_bits, data_terms).to(device)
        self.group_size = group_size
        self.num_terms = num_terms
        self.weight_bits = weight_bits
        l = lstm_layer
        self.termpair = bool(
            termpair and isinstance(l, nn.LSTM) and l.bias and not l.batch_first and
            not l.bidirectional and getattr(l, 'proj_size', 0) == 0 and
            l.weight_ih_l0.dtype == torch.float32 and
            weight_bits <= tq_ops.MAX_CODE_BITS and data_bits <= tq_ops.MAX_CODE_BITS)

        # ih_l0, hh_l0 (the reference overwrites self.w_sf: the hh scale remains)
        names = ('weight_ih_l0', 'weight_hh_l0')
        trd = {}
        for name in names:
            w = getattr(lstm_layer, name)
            sf = _w_sf(w, weight_bits)
            if self.termpair:
                wq, codes = tq_ops.tr_encode(w.detach().contiguous(), sf, weight_bits,
                                             self.group_size, self.num_terms)
                # int32 accumulator bound of the term-pair GEMM, as TRConv2dLayer /
                # TRLinearLayer check it: sum_k |v_w| * max|v_x| (|v_x| <= 2^data_bits)
                if codes.abs().to(torch.int64).sum(1).max().item() << data_bits >= 2**31:
                    self.termpair = False
            else:
                wq, codes = tr_cuda.tr(w, sf, weight_bits, self.group_size,
                                       self.num_terms), None
            trd[name] = (sf, wq, codes)
        for name in names:
            sf, wq, codes = trd[name]
            self.w_sf = sf
            if self.termpair:
                packed, cp, engine, kc = _pack_termpair(codes[:, :, None, None], data_bits,
                                                        weight_bits)
                kch = _kc_chunk(packed, engine, data_bits, cp, 1)
                tag = name[7:9]  # 'ih' / 'hh'
                self.register_buffer('w_codes_' + tag, packed)
                setattr(self, '_tp_' + tag, (cp, self.w_sf, kc, kch))
            setattr(lstm_layer, name, nn.Parameter(wq))

        self.lstm = lstm_layer
        self.lstm.flatten_parameters()
        upper = None
        if self.termpair and l.num_layers > 1:
            # layers >= 1 as their own library LSTM sharing the parameters (kept out of the
            # module tree, so state_dict() and parameters() are the reference's)
            upper = nn.LSTM(l.hidden_size, l.hidden_size, l.num_layers - 1, bias=True).to(device)
            for k in range(1, l.num_layers):
                for p in ('weight_ih', 'weight_hh', 'bias_ih', 'bias_hh'):
                    setattr(upper, '%s_l%d' % (p, k - 1), getattr(l, '%s_l%d' % (p, k)))
            upper.flatten_parameters()
        self.__dict__['_upper'] = upper

    def _tp_linear(self, x, tag, bias):
        cp, sf_w, kc, kch = getattr(self, '_tp_' + tag)
        codes = getattr(self, 'w_codes_' + tag)
        return tq_ops.tr_linear(x, self.input_quant.sf, self.data_bits, self.data_terms, codes,
                                cp, sf_w, bias, 4 * self.lstm.hidden_size, kc, kch)

    def _forward_termpair(self, emb, hidden):
        l = self.lstm
        h0, c0 = hidden
        hq = self.input_quant(h0)  # the reference quantizes every layer's initial state
        cq = self.input_quant(c0)
        T, B, _ = emb.shape
        H = l.hidden_size
        gx = self._tp_linear(emb.contiguous(), 'ih', l.bias_ih_l0).contiguous()  # [T, B, 4H]
        out0 = torch.empty((T, B, H), dtype=emb.dtype, device=emb.device)
        if not self._seq_kernel(B, H):  # per-step launches (TQ_LSTM_SEQ=0, A/B)
            w_hh = l.weight_hh_l0
            c = cq[0].contiguous().clone()
            h = None
            for t in range(T):
                if t == 0:  # TR(h0) x TR(W_hh): term-pair
                    hh = self._tp_linear(h0[0].contiguous(), 'hh', l.bias_hh_l0)
                else:
                    hh = torch.addmm(l.bias_hh_l0, h, w_hh.t())
                tq_native.lstm_cell(gx[t], hh.contiguous(), c, out0[t])
                h = out0[t]
            hn, cn = [out0[T - 1]], [c]
            out = out0
            if self._upper is not None:
                out, (hu, cu) = self._upper(out0, (hq[1:].contiguous(), cq[1:].contiguous()))
                hn += list(hu)
                cn += list(cu)
            return out, (torch.stack(hn), torch.stack(cn))
        # each layer's recurrence in one call (tq_lstm_seq_f32: a fused step kernel per
        # step); layer 0 from TR(h0), TR(c0) with the TR'd W_hh (fp32 on the TR'd values)
        c_last = torch.empty((l.num_layers, B, H), dtype=emb.dtype, device=emb.device)
        if (l.num_layers == 2 and self._upper is not None and
                os.environ.get("TQ_LSTM_WAVE", "1") != "0" and
                os.environ.get("TQ_LSTM_UPPER", "seq") != "miopen" and
                tq_native.lstm_seq2_supported(B, H)):
            # both layers in wavefront order (tq_lstm_seq2_f32): layer 1's step t beside
            # layer 0's step t + 1 in one launch, its input projection inside the step
            out1 = torch.empty((T, B, H), dtype=emb.dtype, device=emb.device)
            tq_native.lstm_seq2(gx, l.weight_hh_l0.contiguous(), l.bias_hh_l0.contiguous(),
                                hq[0].contiguous(), cq[0].contiguous(),
                                l.weight_ih_l1.contiguous(), l.bias_ih_l1.contiguous(),
                                l.weight_hh_l1.contiguous(), l.bias_hh_l1.contiguous(),
                                hq[1].contiguous(), cq[1].contiguous(), out0, out1, c_last[0],
                                c_last[1])
            return out1, (torch.stack([out0[T - 1], out1[T - 1]]), c_last)
        tq_native.lstm_seq(gx, l.weight_hh_l0.contiguous(), l.bias_hh_l0.contiguous(),
                           hq[0].contiguous(), cq[0].contiguous(), out0, c_last[0])
        outs = [out0]
        if self._upper is not None and os.environ.get("TQ_LSTM_UPPER", "seq") == "miopen":
            out, (hu, cu) = self._upper(out0, (hq[1:].contiguous(), cq[1:].contiguous()))
            return out, (torch.cat([out0[T - 1:], hu]), torch.cat([c_last[:1], cu]))
        x = out0
        for k in range(1, l.num_layers):
            # layers >= 1 (weights untouched by the reference): input projection over all
            # steps as one GEMM, then the recurrence in one call
            w_ih = getattr(l, 'weight_ih_l%d' % k)
            gxk = torch.addmm(getattr(l, 'bias_ih_l%d' % k), x.view(T * B, H),
                              w_ih.t()).view(T, B, 4 * H)
            yk = torch.empty((T, B, H), dtype=emb.dtype, device=emb.device)
            tq_native.lstm_seq(gxk, getattr(l, 'weight_hh_l%d' % k).contiguous(),
                               getattr(l, 'bias_hh_l%d' % k).contiguous(),
                               hq[k].contiguous(), cq[k].contiguous(), yk, c_last[k])
            outs.append(yk)
            x = yk
        hn = torch.stack([o[T - 1] for o in outs])
        return x, (hn, c_last)

    @staticmethod
    def _seq_kernel(batch, hidden):
        return (os.environ.get("TQ_LSTM_SEQ", "1") != "0" and
                tq_native.lstm_seq_workspace_bytes(batch, hidden) >= 0)

    def forward(self, emb, hidden):
        if self.termpair and not self.input_quant.tracking and emb.is_cuda:
            return self._forward_termpair(emb, hidden)
        embq = self.input_quant(emb)
        hidden_qs = tuple(self.input_quant(h) for h in hidden)

        return self.lstm(embq, hidden_qs)

    def tracking(self, tracking):
        if not tracking:
            self.input_quant.finish_tracking()
        else:
            self.input_quant.tracking = True
