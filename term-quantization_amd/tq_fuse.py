"""Fused TQ executor for a converted, calibrated ResNet (BasicBlock) model.

The module path (torchvision-style ResNet with TRConv2dLayer, BatchNorm2d, ReLU modules) runs
every op as its own pass over HBM: term-pair conv -> BN -> ReLU -> (+identity -> ReLU) ->
the next layer's activation TR.  This executor runs the same math with each block's ops
folded into the term-pair kernel's epilogue (tq_conv2d_termpair_fused):

  conv1:       codes(x; sf1)   -> TR(relu(bn1(conv1)); sf2) as codes         (no fp32 tensor)
  downsample:  codes(x; sf_d)  -> bn_d(conv_d) fp32                          (the identity)
  conv2:       codes(mid; sf2) -> y = relu(bn2(conv2) + identity) fp32, plus
                                  TR(y; sf of the next block's conv1 / downsample) codes

so between the stem and the classifier only the term-pair kernels touch HBM.  BatchNorm is
folded per channel in fp64 (eval mode: y*gamma/sqrt(var+eps) + beta - mean*gamma/sqrt(..)),
the sum rounds to fp32 once, the residual add and ReLU are fp32 as in the module path, and
each activation code is TR of exactly that fp32 value (tr_layer.py:96-99), so the executor
matches the module path to fp32 rounding of the BN (DESIGN.md "Fused executor").
"""
import os

import numpy as np
import torch
import torch.nn as nn

import tq_native
import tq_ops
import tr_layer


def _bn_affine(bn):
    """An eval BatchNorm as an fp32 per-channel affine (scale, shift) for tq_act_encode_act."""
    a = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
    return (a.float().contiguous(),
            (bn.bias.detach().double() - bn.running_mean.detach().double() * a).float()
            .contiguous())


def _fold_bn(layer, bn):
    """Per-channel (scale, shift) in fp64: bn(acc * s + bias) == acc * scale + shift."""
    dev = layer.w_codes.device
    s = float(np.float32(layer.input_quant.sf)) * float(np.float32(layer.w_sf))
    bias = (layer.conv.bias.detach().double() if layer.conv.bias is not None
            else torch.zeros(layer.conv.out_channels, dtype=torch.float64, device=dev))
    if bn is None:
        return (torch.full_like(bias, s), bias.clone())
    a = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
    scale = s * a
    shift = (bias - bn.running_mean.detach().double()) * a + bn.bias.detach().double()
    return scale.contiguous(), shift.contiguous()


class _Conv(object):
    """One TRConv2dLayer prepared for the fused kernel."""

    def __init__(self, layer, bn, nonneg=False):
        if not isinstance(layer, tr_layer.TRConv2dLayer) or not layer.termpair:
            raise ValueError("fused executor needs term-pair TRConv2dLayer convolutions")
        if layer.input_quant.tracking:
            raise ValueError("calibrate first: set_tr_tracking(model, False)")
        c = layer.conv
        self.layer = layer
        self.cout = c.out_channels
        self.kh, self.kw = c.kernel_size
        self.stride, self.padding, self.dilation = c.stride, c.padding, c.dilation
        self.cp_in = layer.act_channels
        self.quant = (layer.input_quant.sf, layer.data_bits, layer.data_terms)
        self.bn = bn
        self.scale, self.shift = _fold_bn(layer, bn)
        self.code_dtype = layer.w_codes.dtype   # int16 (VALU engine) / float16 (MFMA engine)
        # nonneg: the caller guarantees the input codes are TR of a ReLU output (>= 0), so
        # the wider non-negative exactness windows hold; otherwise the general ones
        self.nonneg = bool(nonneg)
        self.kc_steps = layer.kc_steps_nonneg if nonneg else layer.kc_steps
        self.kc_chunk = layer.kc_chunk_nonneg if nonneg else layer.kc_chunk
        if self.cout % 4:
            raise ValueError("fused epilogue needs Cout % 4 == 0")

    def out_hw(self, h, w):
        return (tq_ops.conv_out_size(h, self.kh, self.stride[0], self.padding[0],
                                     self.dilation[0]),
                tq_ops.conv_out_size(w, self.kw, self.stride[1], self.padding[1],
                                     self.dilation[1]))

    def fusable_downsample(self, down):
        """True when ``down`` (a block's 1x1 pad-0 downsample) can run as the second
        accumulation phase of this conv (tq_conv_epilogue.ds_*): MFMA codes on both, 64-code
        channel chunks, and a downsample whose fp32 sums need no flush.  Opt-in
        (TQ_FUSE_DS=1): the phase runs on the direct engine only, and at batch 256 the fused
        layer-2 conv took as long as conv2 + downsample apart (190.8 vs 158 + 31 us) while the
        layer-3/4 conv2s lost the input-patch engine (188/198 vs ~121/~102 us + ~15 us;
        profiles/r02b_summary.json)."""
        nsteps = down.layer.w_codes.shape[1] // 64
        return (os.environ.get("TQ_FUSE_DS", "0") == "1" and
                self.code_dtype == torch.float16 and down.code_dtype == torch.float16 and
                self.cp_in % 64 == 0 and down.cp_in % 64 == 0 and
                (down.kh, down.kw) == (1, 1) and tuple(down.padding) == (0, 0) and
                tuple(down.dilation) == (1, 1) and down.stride[0] == down.stride[1] and
                down.layer.w_codes.shape[1] == down.cp_in and
                (down.kc_steps == 0 or down.kc_steps >= nsteps) and
                down.cout == self.cout)

    def __call__(self, codes, out=None, residual=None, relu=False, next_a=None, next_b=None,
                 downsample=None):
        """``downsample`` = (_Conv, its input codes): computed in this launch as a second
        accumulation phase, its identity added in place of ``residual``."""
        for nxt in (next_a, next_b):
            if nxt is not None and nxt.nonneg and not (relu is True or relu in (1, 6)):
                raise ValueError("a consumer with non-negative windows needs ReLU'd codes")
        n, h, w, _ = codes.shape
        ho, wo = self.out_hw(h, w)
        dev = codes.device
        ca = cb = None
        if next_a is not None:
            ca = torch.empty((n, ho, wo, next_a.cp_in), dtype=next_a.code_dtype, device=dev)
        if next_b is not None:
            cb = torch.empty((n, ho, wo, next_b.cp_in), dtype=next_b.code_dtype, device=dev)
        if out is True:
            out = torch.empty((n, self.cout, ho, wo), dtype=torch.float32, device=dev,
                              memory_format=torch.channels_last)
        res = None
        if residual is not None:
            res = residual if residual.is_contiguous(memory_format=torch.channels_last) \
                else residual.contiguous(memory_format=torch.channels_last)
        cin = self.layer.conv.in_channels
        ws = tq_native.conv2d_workspace(n * ho * wo, self.cout, dev)
        # algorithmic HBM bytes: each tensor the launch reads or writes, once
        nbytes = codes.numel() * codes.element_size() + \
            self.layer.w_codes.numel() * self.layer.w_codes.element_size() + \
            sum(t.numel() * t.element_size() for t in (out, res, ca, cb) if t is not None)
        work = n * ho * wo * self.cout * cin * self.kh * self.kw
        ds = None
        if downsample is not None:
            down, dcodes = downsample
            if res is not None:
                raise ValueError("a fused downsample replaces the residual")
            if dcodes.shape[-1] != down.cp_in or not self.fusable_downsample(down):
                raise ValueError("downsample cannot be fused into this conv")
            ds = (dcodes, down.layer.w_codes, down.stride[0], down.scale, down.shift)
            nbytes += dcodes.numel() * dcodes.element_size() + \
                down.layer.w_codes.numel() * down.layer.w_codes.element_size()
            work += n * ho * wo * self.cout * down.layer.conv.in_channels
        tq_ops._launch(
            "conv2d_termpair", work,
            lambda: tq_native.conv2d_termpair_fused(
                codes, self.layer.w_codes, self.cout, self.kh, self.kw, self.stride,
                self.padding, self.dilation, ho, wo, out=out, ch_scale=self.scale,
                ch_shift=self.shift, residual=res, relu=relu, codes_a=ca,
                quant_a=next_a.quant if next_a else None, codes_b=cb,
                quant_b=next_b.quant if next_b else None, workspace=ws,
                kc_steps=self.kc_steps, kc_chunk=self.kc_chunk, downsample=ds), nbytes)
        return out, ca, cb


def _same_codes(a, b):
    """True when two consumers of one activation would get identical codes: same TR
    parameters (sf, data bits, data terms), code format and channel padding.  A block's conv1
    and downsample read the same tensor, so their calibrated quantizers agree and the
    downsample reuses conv1's codes instead of a second encode + store."""
    return ([float(v) for v in a.quant] == [float(v) for v in b.quant] and
            a.code_dtype == b.code_dtype and a.cp_in == b.cp_in)


class _Block(object):
    def __init__(self, block):
        # every code tensor of the executor is TR of a ReLU output: the stem and every conv
        # epilogue that emits codes apply ReLU first (forward() asserts relu wherever codes are
        # produced), so all three convs take the non-negative windows
        self.conv1 = _Conv(block.conv1, block.bn1, nonneg=True)
        self.conv2 = _Conv(block.conv2, block.bn2, nonneg=True)
        self.down = None
        if block.downsample is not None:
            self.down = _Conv(block.downsample[0], block.downsample[1], nonneg=True)


def _pool_params(mp):
    k, s, p = mp.kernel_size, mp.stride, mp.padding
    if any(isinstance(v, tuple) for v in (k, s, p)) or mp.dilation != 1 or mp.ceil_mode:
        return None
    return int(k), int(s), int(p)


class FusedResNet(nn.Module):
    """Inference executor over a converted + calibrated torchvision-style ResNet.

    ``stem="exact"`` (default) runs conv1 + bn1 + relu + maxpool + the first codes as one
    kernel whose conv is split-fp16 on the matrix cores, plus the exact fix-up of every output
    whose code the split's error could change, so the codes are those of the correctly rounded
    fp32 conv; ``stem="fused"`` is that kernel without the fix-up (on the bench
    batch its codes are closer to the correctly rounded conv's than torch's own fp32 convs
    are, 7 % faster in the bench); ``stem="fp32"`` keeps
    torch's fp32 conv1 (MIOpen's true fp32: gfx950 has no TF32 / xf32) and runs only BN + ReLU
    + max-pool + codes in one kernel -- the reference's arithmetic for the stem conv
    (bench.py --stem)."""

    def __init__(self, qmodel, stem="exact"):
        super(FusedResNet, self).__init__()
        if stem not in ("fused", "exact", "fp32"):
            raise ValueError("stem must be 'fused', 'exact' or 'fp32'")
        self.qmodel = qmodel
        self.blocks = []
        for layer in (qmodel.layer1, qmodel.layer2, qmodel.layer3, qmodel.layer4):
            for block in layer:
                self.blocks.append(_Block(block))
        # stem tail: eval BN as an fp32 per-channel affine for the fused pool+encode pass
        bn = qmodel.bn1
        self.pool = _pool_params(qmodel.maxpool)
        a = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
        self.stem_scale = a.float().contiguous()
        self.stem_shift = (bn.bias.detach().double() -
                           bn.running_mean.detach().double() * a).float().contiguous()
        self.fuse_stem = (self.pool is not None and not bn.training and
                          bn.num_features % 8 == 0)
        # the whole stem (conv + BN + ReLU + pool + codes) in one kernel when it is the
        # torchvision shape: conv 7x7/2 pad 3, 3 -> 64, no bias; pool 3x3/2 pad 1
        c1 = qmodel.conv1
        self.stem_w = None
        self.stem_exact = None
        if (stem in ("fused", "exact") and self.fuse_stem and self.pool == (3, 2, 1) and
                isinstance(c1, nn.Conv2d)
                and type(c1) is nn.Conv2d and c1.in_channels == 3 and c1.out_channels == 64
                and c1.kernel_size == (7, 7) and c1.stride == (2, 2) and c1.padding == (3, 3)
                and c1.dilation == (1, 1) and c1.groups == 1 and c1.bias is None
                and c1.weight.dtype == torch.float32):
            try:
                self.stem_w = tq_ops.pack_stem_weight(c1.weight)
            except RuntimeError:  # weights outside the fp16 split's range: unfused stem
                self.stem_w = None
            if self.stem_w is not None and stem == "exact":
                self.stem_exact = tq_ops.pack_stem_exact(c1.weight)

    def _stem_fused(self, x, first):
        n, _, h, w = x.shape
        out = torch.empty((n, 64, h // 4, w // 4), dtype=torch.float32, device=x.device,
                          memory_format=torch.channels_last)
        codes = torch.empty((n, h // 4, w // 4, first.conv1.cp_in),
                            dtype=first.conv1.code_dtype, device=x.device)
        codes_down = None
        shared = first.down is not None and _same_codes(first.conv1, first.down)
        if first.down is not None and not shared:
            codes_down = torch.empty((n, h // 4, w // 4, first.down.cp_in),
                                     dtype=first.down.code_dtype, device=x.device)
        ws = None
        if self.stem_exact is not None:
            ws = tq_native.stem_workspace(n, h, w, x.device)
        # work = the stem conv's fp32 MACs (7x7x3 per output of the 64 x H/2 x W/2 conv)
        tq_ops._launch(
            "stem_conv_pool", n * 64 * (h // 2) * (w // 2) * 147,
            lambda: tq_native.stem_conv_pool_encode(
                x, self.stem_w, self.stem_scale, self.stem_shift, out, codes_a=codes,
                quant_a=first.conv1.quant, codes_b=codes_down,
                quant_b=first.down.quant if codes_down is not None else None,
                exact=self.stem_exact, workspace=ws))
        return out, codes, (codes if shared else codes_down)

    def _stem(self, x):
        m = self.qmodel
        first = self.blocks[0]
        n, _, h, w = x.shape
        if self.stem_w is not None and h % 4 == 0 and w % 4 == 0 and w // 4 <= 84:
            return self._stem_fused(x, first)
        if not self.fuse_stem:
            x = m.maxpool(m.relu(m.bn1(m.conv1(x)))).contiguous(
                memory_format=torch.channels_last)
            codes = torch.empty((x.shape[0], x.shape[2], x.shape[3], first.conv1.cp_in),
                                dtype=first.conv1.code_dtype, device=x.device)
            tq_ops._launch("act_encode", 4 * x.numel() + 2 * codes.numel(),
                           lambda: tq_native.act_encode(x, True, *first.conv1.quant, codes))
            codes_down = None
            if first.down is not None:
                codes_down = torch.empty((x.shape[0], x.shape[2], x.shape[3],
                                          first.down.cp_in), dtype=first.down.code_dtype,
                                         device=x.device)
                tq_native.act_encode(x, True, *first.down.quant, codes_down)
            return x, codes, codes_down
        y = m.conv1(x).contiguous(memory_format=torch.channels_last)
        n, c, h, w = y.shape
        k, s, p = self.pool
        ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        out = torch.empty((n, c, ho, wo), dtype=torch.float32, device=y.device,
                          memory_format=torch.channels_last)
        codes = torch.empty((n, ho, wo, first.conv1.cp_in), dtype=first.conv1.code_dtype,
                            device=y.device)
        codes_down = None
        if first.down is not None:
            codes_down = torch.empty((n, ho, wo, first.down.cp_in), dtype=first.down.code_dtype,
                                     device=y.device)
        tq_ops._launch(
            "stem_pool_encode", 4 * y.numel() + 4 * out.numel() + 2 * codes.numel(),
            lambda: tq_native.bn_relu_maxpool_encode(
                y, self.stem_scale, self.stem_shift, k, s, p, out, codes_a=codes,
                quant_a=first.conv1.quant, codes_b=codes_down,
                quant_b=first.down.quant if first.down is not None else None))
        return out, codes, codes_down

    @torch.no_grad()
    def forward(self, x, capture=None):
        """Logits of a batch.  ``capture`` (a list, tests only) receives one record per
        term-pair conv -- {"name", "conv", "codes_in", "residual", "out", "codes_a",
        "codes_b"} -- plus a "stem" record, and makes every conv also store its fp32 output
        (the epilogue computes it either way; the codes are identical)."""
        res = []
        for _ in self._steps(x, capture, res):
            pass
        return res[0]

    @torch.no_grad()
    def forward_streams(self, x, streams):
        """Logits of a batch split into len(streams) image chunks, one chunk per HIP stream.
        Each chunk runs the same kernels as forward() on its images (every kernel is
        per-image independent, so the logits are bit-identical); the launches are issued
        layer by layer, round-robin over the streams, so while one chunk's kernel drains
        its last workgroups the other chunk's kernel fills the idle CUs."""
        if len(streams) <= 1:
            return self.forward(x)
        cur = torch.cuda.current_stream(x.device)
        chunks = x.chunk(len(streams))
        gens, res = [], []
        for s, xc in zip(streams, chunks):
            s.wait_stream(cur)
            r = []
            res.append(r)
            gens.append(self._steps(xc, None, r))
        # TQ_STREAM_LAG=L: chunk j starts j * L launches late, so the streams run different
        # layers side by side (A/B option; 0 = lockstep round-robin)
        lag = int(os.environ.get("TQ_STREAM_LAG", "0"))
        live = list(range(len(gens)))
        rnd = 0
        while live:
            nxt = []
            for j in live:
                if rnd < j * lag:
                    nxt.append(j)
                    continue
                with torch.cuda.stream(streams[j]):
                    if next(gens[j], StopIteration) is not StopIteration:
                        nxt.append(j)
            live = nxt
            rnd += 1
        capturing = torch.cuda.is_current_stream_capturing()
        for s, xc, r in zip(streams, chunks, res):
            cur.wait_stream(s)
            if not capturing:  # (a captured graph keeps its private pool alive)
                xc.record_stream(s)
                r[0].record_stream(cur)
        return torch.cat([r[0] for r in res])

    def _steps(self, x, capture, result):
        """forward() as a generator: yields after each kernel launch (the block index after a
        block's last conv, else None); the logits end up in result[0]."""
        m = self.qmodel
        keep = capture is not None
        x = x.contiguous(memory_format=torch.channels_last)
        x, codes, codes_down = self._stem(x)
        yield
        if keep:
            capture.append({"name": "stem", "out": x, "codes_a": codes, "codes_b": codes_down})
        for i, b in enumerate(self.blocks):
            nxt = self.blocks[i + 1] if i + 1 < len(self.blocks) else None
            y1, mid, _ = b.conv1(codes, out=True if keep else None, relu=True, next_a=b.conv2)
            yield
            if keep:
                capture.append({"name": "block%d.conv1" % i, "conv": b.conv1, "codes_in": codes,
                                "residual": None, "out": y1, "codes_a": mid, "codes_b": None})
            fuse_ds = b.down is not None and b.conv2.fusable_downsample(b.down)
            if b.down is not None and (not fuse_ds or keep):
                # (capture runs it separately as well, to record the identity it must equal)
                identity, _, _ = b.down(codes_down, out=True)
                yield
                if keep:
                    capture.append({"name": "block%d.downsample" % i, "conv": b.down,
                                    "codes_in": codes_down, "residual": None, "out": identity,
                                    "codes_a": None, "codes_b": None})
            elif b.down is None:
                identity = x
            next_b = nxt.down if nxt is not None and nxt.down is not None else None
            shared = next_b is not None and _same_codes(nxt.conv1, next_b)
            # a block followed by a downsampling block: its fp32 output is nobody's residual
            # (the next identity is the downsample conv's), so only its codes are written
            cin = mid
            x, codes, codes_down = b.conv2(
                mid, out=True if (next_b is None or keep) else None,
                residual=None if fuse_ds else identity,
                relu=True, next_a=nxt.conv1 if nxt else None,
                next_b=None if shared else next_b,
                downsample=(b.down, codes_down) if fuse_ds else None)
            yield i  # block i done
            if shared:
                codes_down = codes
            if keep:
                capture.append({"name": "block%d.conv2" % i, "conv": b.conv2, "codes_in": cin,
                                "residual": identity, "out": x, "codes_a": codes,
                                "codes_b": codes_down})
        x = m.avgpool(x)
        x = torch.flatten(x, 1)
        result.append(m.fc(x))


# ---------------------------------------------------------------------------------------
# MobileNet-V2 (torchvision topology, cnn_models/mobilenet.py): inverted-residual blocks
#   expand 1x1 -> BN -> ReLU6 -> dw 3x3 -> BN -> ReLU6 -> project 1x1 -> BN (+ identity)
# with every BN / ReLU6 / residual add and the next layer's activation TR in the producing
# kernel's epilogue (term-pair convs: tq_conv2d_termpair_f16 relu = 2; depthwise:
# tq_dwconv2d_termpair_fused), so between the stem and the classifier only the term-pair
# kernels touch HBM -- fp32 tensors only where a residual or the pooling needs them.


def _run_chunks(streams, codes, xin, y, body):
    """Run body(codes, xin, y) generators over image chunks of a batch, one chunk per HIP
    stream, one launch per stream in turn (FusedResNet.forward_streams): every launch is
    per-image independent, so the chunks compute exactly what one launch over the batch
    does.  ``y`` (the head conv's output) is written chunk by chunk in place."""
    cur = torch.cuda.current_stream(codes.device)
    n = len(streams)
    parts = [codes.chunk(n), xin.chunk(n) if xin is not None else [None] * n, y.chunk(n)]
    gens = []
    for s, c, xi, yi in zip(streams, *parts):
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            gens.append(body(c, xi, yi))
    live = list(range(len(gens)))
    while live:
        nxt = []
        for j in live:
            with torch.cuda.stream(streams[j]):
                if next(gens[j], StopIteration) is not StopIteration:
                    nxt.append(j)
        live = nxt
    capturing = torch.cuda.is_current_stream_capturing()
    for s, c, xi in zip(streams, parts[0], parts[1]):
        cur.wait_stream(s)
        if not capturing:  # (a captured graph keeps its private pool alive)
            c.record_stream(s)
            if xi is not None:
                xi.record_stream(s)
            y.record_stream(s)


class _Codes(object):
    """What a producing epilogue needs to know about a consuming TR layer."""

    def __init__(self, layer, code_dtype, nonneg):
        self.quant = (layer.input_quant.sf, layer.data_bits, layer.data_terms)
        self.cp_in = layer.act_channels
        self.code_dtype = code_dtype
        self.nonneg = nonneg


class _DwConv(object):
    """A depthwise TRConv2dLayer (mode "depthwise") + its BN + ReLU6, for the fused kernel."""

    def __init__(self, layer, bn):
        if not isinstance(layer, tr_layer.TRConv2dLayer) or layer.mode != "depthwise":
            raise ValueError("fused executor needs depthwise term-pair TRConv2dLayers")
        if layer.input_quant.tracking:
            raise ValueError("calibrate first: set_tr_tracking(model, False)")
        c = layer.conv
        # Conv2dStaticSamePadding (EfficientNet): taps outside the input read 0, so the
        # (top, left) pad plus the padded output size express the asymmetric padding
        self.pad_tblr = tq_ops.static_padding(c)
        self.layer = layer
        self.c = c.out_channels
        self.kh, self.kw = c.kernel_size
        self.stride, self.padding, self.dilation = c.stride, c.padding, c.dilation
        self.bn = bn
        self.scale, self.shift = _fold_bn(layer, bn)
        self.consumer = _Codes(layer, torch.int16, False)

    def out_hw(self, h, w):
        top, bottom, left, right = self.pad_tblr
        return (tq_ops.conv_out_size(h + top + bottom, self.kh, self.stride[0],
                                     self.padding[0], self.dilation[0]),
                tq_ops.conv_out_size(w + left + right, self.kw, self.stride[1],
                                     self.padding[1], self.dilation[1]))

    def __call__(self, codes, nxt, out=False, act=6):
        """BN + ``act`` (6: ReLU6, "swish") in the epilogue; ``nxt`` (a _Codes / _Conv) gets
        its input codes unless None (then ``out`` must be set)."""
        n, h, w, cp = codes.shape
        ho, wo = self.out_hw(h, w)
        dev = codes.device
        y = (torch.empty((n, self.c, ho, wo), dtype=torch.float32, device=dev,
                         memory_format=torch.channels_last) if out else None)
        nc = None
        if nxt is not None:
            nc = torch.empty((n, ho, wo, nxt.cp_in), dtype=nxt.code_dtype, device=dev)
            if nxt.cp_in != cp:
                raise ValueError("depthwise output codes must have the input's channel padding")
        w_codes = self.layer.w_codes
        nbytes = codes.numel() * 2 + w_codes.numel() * 4 + \
            sum(t.numel() * t.element_size() for t in (y, nc) if t is not None)
        pad_tl = (self.pad_tblr[0] + self.padding[0], self.pad_tblr[2] + self.padding[1])
        tq_ops._launch(
            "dwconv2d_termpair", n * ho * wo * self.c * self.kh * self.kw,
            lambda: tq_native.dwconv2d_termpair_fused(
                codes, self.c, w_codes, self.kh, self.kw, self.stride, pad_tl,
                self.dilation, ho, wo, self.scale, self.shift, act, out=y, next_codes=nc,
                quant=nxt.quant if nxt is not None else None), nbytes)
        return y, nc


class _InvRes(object):
    def __init__(self, block):
        mods = list(block.conv)
        self.use_res = block.use_res_connect
        if len(mods) == 3:  # expand ratio 1: dw, project conv, BN
            self.expand = None
            dw, proj, bn = mods[0], mods[1], mods[2]
        else:
            self.expand = _Conv(mods[0][0], mods[0][1], nonneg=False)
            dw, proj, bn = mods[1], mods[2], mods[3]
        self.dw = _DwConv(dw[0], dw[1])
        # the project conv's input codes are TR of a ReLU6 output: non-negative windows
        self.project = _Conv(proj, bn, nonneg=True)

    def first_consumer(self):
        """The consumer of this block's input codes: the expand conv, else the dw conv."""
        return self.expand if self.expand is not None else self.dw.consumer

    def out_hw(self, h, w):
        return self.dw.out_hw(h, w)  # (the 1x1 convs keep the size)


class FusedMobileNetV2(nn.Module):
    """Inference executor over a converted + calibrated MobileNet-V2 (cnn_models.mobilenet_v2
    with depthwise layers at (16, 1, 16) and the rest term-pair, cnn_models/__init__.py:31-58).
    The stem conv (never converted: an fp32 torch conv, cnn_models/__init__.py:34-36) and the
    classifier stay torch."""

    def __init__(self, qmodel):
        super(FusedMobileNetV2, self).__init__()
        from cnn_models.mobilenet import InvertedResidual
        self.qmodel = qmodel
        feats = list(qmodel.features)
        self.stem = feats[0]
        self.blocks = [_InvRes(b) for b in feats[1:-1]]
        if not all(isinstance(b, InvertedResidual) for b in feats[1:-1]):
            raise ValueError("not a torchvision-style MobileNet-V2")
        last = feats[-1]
        self.last = _Conv(last[0], last[1], nonneg=False)
        # stem: torch conv, then BN + ReLU6 + the first block's codes in one pass
        self.stem_affine = None
        if (len(self.stem) == 3 and isinstance(self.stem[1], nn.BatchNorm2d) and
                isinstance(self.stem[2], nn.ReLU6) and not self.stem[1].training):
            self.stem_affine = _bn_affine(self.stem[1])

    @torch.no_grad()
    def forward(self, x, capture=None):
        """Logits of a batch.  ``capture`` (a list, tests only) receives one record per
        term-pair / depthwise layer: {"name", "kind", "conv", "codes_in", "residual", "out",
        "codes_out"}; capture mode also stores every fp32 output."""
        codes, xin = self._stem(x, capture)
        y = self._head_out(codes)
        for _ in self._body(codes, xin, y, capture):
            pass
        return self._classify(y)

    @torch.no_grad()
    def forward_streams(self, x, streams):
        """forward() with the blocks of len(streams) image chunks on their own HIP streams,
        launched layer by layer round-robin (as FusedResNet.forward_streams): one chunk's
        short launches fill the CUs the other's leave idle.  The torch stem conv and the
        classifier run on the whole batch (their library kernels may pick another algorithm
        for another batch size), so the logits are bit-identical to forward()'s."""
        codes, xin = self._stem(x, None)
        y = self._head_out(codes)
        _run_chunks(streams, codes, xin, y, self._body)
        return self._classify(y)

    def _head_out(self, codes):
        n, h, w, _ = codes.shape
        for b in self.blocks:
            h, w = b.out_hw(h, w)
        return torch.empty((n, self.last.cout, h, w), dtype=torch.float32, device=codes.device,
                           memory_format=torch.channels_last)

    def _classify(self, y):
        y = nn.functional.adaptive_avg_pool2d(y, 1).reshape(y.shape[0], -1)
        return self.qmodel.classifier(y)

    def _stem(self, x, capture):
        keep = capture is not None
        x = x.contiguous(memory_format=torch.channels_last)
        first = self.blocks[0].first_consumer()
        if self.stem_affine is not None:
            z = self.stem[0](x).contiguous(memory_format=torch.channels_last)
            codes = torch.empty((z.shape[0], z.shape[2], z.shape[3], first.cp_in),
                                dtype=first.code_dtype, device=x.device)
            y0 = torch.empty_like(z) if (keep or self.blocks[0].use_res) else None
            tq_ops._launch("act_encode_act", 4 * z.numel() + 2 * codes.numel(),
                           lambda: tq_native.act_encode_act(z, *first.quant, codes, act=6,
                                                            out=y0, affine=self.stem_affine))
        else:
            y0 = self.stem(x).contiguous(memory_format=torch.channels_last)  # conv, BN, ReLU6
            codes = torch.empty((y0.shape[0], y0.shape[2], y0.shape[3], first.cp_in),
                                dtype=first.code_dtype, device=x.device)
            tq_ops._launch("act_encode", 4 * y0.numel() + 2 * codes.numel(),
                           lambda: tq_native.act_encode(y0, True, *first.quant, codes))
        if keep:
            capture.append({"name": "stem", "kind": "stem", "out": y0, "codes_out": codes,
                            "quant": first.quant})
        return codes, y0

    def _body(self, codes, xin, y, capture=None):
        """The blocks and the last conv (into ``y``) as a generator: yields after each
        launch."""
        keep = capture is not None
        for i, b in enumerate(self.blocks):
            nxt = self.blocks[i + 1] if i + 1 < len(self.blocks) else None
            if b.expand is not None:
                h, hcodes, _ = b.expand(codes, out=True if keep else None, relu=6,
                                        next_a=b.dw.consumer)
                yield
                if keep:
                    capture.append({"name": "block%d.expand" % i, "kind": "conv",
                                    "conv": b.expand, "codes_in": codes, "residual": None,
                                    "out": h, "codes_out": hcodes, "relu": 6})
            else:
                hcodes = codes
            d, pcodes = b.dw(hcodes, b.project, out=keep)
            yield
            if keep:
                capture.append({"name": "block%d.dw" % i, "kind": "dw", "conv": b.dw,
                                "codes_in": hcodes, "residual": None, "out": d,
                                "codes_out": pcodes, "relu": 6})
            consumer = nxt.first_consumer() if nxt is not None else self.last
            need_out = keep or (nxt is not None and nxt.use_res)
            xout, codes, _ = b.project(pcodes, out=True if need_out else None,
                                       residual=xin if b.use_res else None, relu=False,
                                       next_a=consumer)
            yield
            if keep:
                capture.append({"name": "block%d.project" % i, "kind": "conv",
                                "conv": b.project, "codes_in": pcodes,
                                "residual": xin if b.use_res else None, "out": xout,
                                "codes_out": codes, "relu": 0})
            xin = xout
        self.last(codes, out=y, relu=6)
        yield
        if keep:
            capture.append({"name": "last", "kind": "conv", "conv": self.last,
                            "codes_in": codes, "residual": None, "out": y, "codes_out": None,
                            "relu": 6})


# ---------------------------------------------------------------------------------------
# EfficientNet-b0 (efficientnet_pytorch topology, cnn_models/efficientnet.py): MBConv blocks
#   [expand 1x1 -> BN -> swish] -> dw kxk (static same padding) -> BN -> swish
#   -> squeeze-excite: x * sigmoid(se_expand(swish(se_reduce(avgpool(x)))))
#   -> project 1x1 -> BN (+ identity)
# The expand conv's epilogue applies BN + swish and writes the dw conv's codes (the direct
# engine's swish instantiation: a runtime swish branch in the shared term-pair epilogue cost
# the ResNet/MobileNet engines scratch); the dw kernel applies
# BN + swish and writes the fp32 tensor the squeeze-excite branch pools; the gate and the
# project conv's input TR are one pass (tq_act_encode_act with the gate); the project
# conv's epilogue adds BN and the identity and writes the next block's codes.  The squeeze-
# excite convs themselves (1x1 on [N, C, 1, 1], 16-bit weights: the module's term-pair
# "wide" kernel) and the pooling stay module calls: a few KB per image.


def _se_plan(block):
    """tq_native.se_gate arguments of an MBConv block's squeeze-excite convs, or None when
    they are not the calibrated 1x1 "wide" TRConv2dLayers the fused kernel covers."""
    convs = (getattr(block, "_se_reduce", None), getattr(block, "_se_expand", None))
    for m in convs:
        if not isinstance(m, tr_layer.TRConv2dLayer) or getattr(m, "mode", None) != "wide":
            return None
        c = m.conv
        if (c.kernel_size != (1, 1) or c.stride != (1, 1) or c.groups != 1 or
                any(tq_ops.static_padding(c)) or c.padding != (0, 0) or
                m.input_quant.tracking or m.data_bits > 14):
            return None
    r, e = convs
    cse, cin = r.conv.out_channels, r.conv.in_channels
    if e.conv.in_channels != cse or e.conv.out_channels != cin:
        return None
    if tuple(r.w_codes.shape) != (cse, tq_ops.act_channels(cin)) or \
            tuple(e.w_codes.shape) != (cin, tq_ops.act_channels(cse)):
        return None

    def conv_args(m, w):
        scale = float(np.float32(m.input_quant.sf)) * float(np.float32(m.w_sf))
        bias = m.conv.bias.detach().float().contiguous() if m.conv.bias is not None else None
        quant = (m.input_quant.sf, m.data_bits, m.data_terms)
        return w, scale, bias, quant
    # the expand conv's codes k-major ([Cse][C]): the kernel's lanes run along C
    w_e_t = e.w_codes[:, :cse].t().contiguous()
    return {"cse": cse, "args": conv_args(r, r.w_codes.contiguous()) + conv_args(e, w_e_t)}


def _conv_out_static(conv, h, w):
    top, bottom, left, right = tq_ops.static_padding(conv.conv)
    c = conv.conv
    return (tq_ops.conv_out_size(h + top + bottom, c.kernel_size[0], c.stride[0], c.padding[0],
                                 c.dilation[0]),
            tq_ops.conv_out_size(w + left + right, c.kernel_size[1], c.stride[1], c.padding[1],
                                 c.dilation[1]))


class _MBConv(object):
    def __init__(self, block):
        self.block = block
        self.expand = None
        for conv in (getattr(block, "_expand_conv", None), block._project_conv):
            if conv is not None and any(tq_ops.static_padding(conv.conv)):
                raise ValueError("1x1 convs of an MBConv block have no padding")
        if block.expand_ratio != 1:
            # its input is a block output (no activation): general exactness windows
            self.expand = _Conv(block._expand_conv, block._bn0, nonneg=False)
        self.dw = _DwConv(block._depthwise_conv, block._bn1)
        self.has_se = block.has_se
        # the project conv's input is swish(...) * gate: signed, general windows
        self.project = _Conv(block._project_conv, block._bn2, nonneg=False)
        self.use_res = (block.id_skip and block.stride == 1 and
                        block.input_filters == block.output_filters)
        self.se = _se_plan(block) if self.has_se else None

    def first_consumer(self):
        return self.expand if self.expand is not None else self.dw.consumer

    def out_hw(self, h, w):
        return self.dw.out_hw(h, w)  # (the 1x1 convs keep the size)

    def gate(self, d):
        """sigmoid(se_expand(swish(se_reduce(avgpool(d))))) as fp32 [N, C]: torch's pooling,
        then the fused squeeze-excite kernel (tq_se_gate_f32: both term-pair convs, swish and
        sigmoid in one launch, bit-identical to the module calls) when the block's convs are
        the "wide" TRConv2dLayers it covers (TQ_SE_FUSED=0: the module calls)."""
        b = self.block
        x_sq = nn.functional.adaptive_avg_pool2d(d, 1)
        if self.se is not None and os.environ.get("TQ_SE_FUSED", "1") != "0":
            n, c = d.shape[0], d.shape[1]
            g = torch.empty((n, c), dtype=torch.float32, device=d.device)
            tq_ops._launch("se_gate", n * c * 2 * self.se["cse"],
                           lambda: tq_native.se_gate(x_sq.reshape(n, c).contiguous(),
                                                     *self.se["args"], g))
            return g
        x_sq = b._se_expand(b._swish(b._se_reduce(x_sq)))
        return torch.sigmoid(x_sq).reshape(d.shape[0], d.shape[1]).contiguous()


class FusedEfficientNet(nn.Module):
    """Inference executor over a converted + calibrated EfficientNet-b0 (cnn_models.
    efficientnet_b0 with depthwise and squeeze-excite convs at (16, 1, 16) and the rest
    term-pair, cnn_models/__init__.py:31-58).  The stem conv (never converted) and the
    classifier stay torch."""

    def __init__(self, qmodel):
        super(FusedEfficientNet, self).__init__()
        from cnn_models.efficientnet import MBConvBlock
        self.qmodel = qmodel
        if not all(isinstance(b, MBConvBlock) for b in qmodel._blocks):
            raise ValueError("not an efficientnet_pytorch-style EfficientNet")
        self.blocks = [_MBConv(b) for b in qmodel._blocks]
        self.head = _Conv(qmodel._conv_head, qmodel._bn1, nonneg=False)
        # stem: torch conv, then BN + swish + the first block's codes in one pass
        self.stem_affine = None if qmodel._bn0.training else _bn_affine(qmodel._bn0)

    @torch.no_grad()
    def forward(self, x, capture=None):
        """Logits of a batch.  ``capture`` (a list, tests only) receives one record per
        term-pair / depthwise layer: {"name", "kind", "conv", "codes_in", "residual", "out",
        "codes_out", "act", "gate"}; capture mode also stores every fp32 output."""
        codes, xin = self._stem(x, capture)
        y = self._head_out(codes)
        for _ in self._body(codes, xin, y, capture):
            pass
        return self._classify(y)

    @torch.no_grad()
    def forward_streams(self, x, streams):
        """forward() with the blocks of len(streams) image chunks on their own HIP streams
        (FusedMobileNetV2.forward_streams); bit-identical logits."""
        codes, xin = self._stem(x, None)
        y = self._head_out(codes)
        _run_chunks(streams, codes, xin, y, self._body)
        return self._classify(y)

    def _head_out(self, codes):
        n, h, w, _ = codes.shape
        for b in self.blocks:
            h, w = b.out_hw(h, w)
        return torch.empty((n, self.head.cout, h, w), dtype=torch.float32, device=codes.device,
                           memory_format=torch.channels_last)

    def _classify(self, y):
        m = self.qmodel
        y = m._avg_pooling(m._swish(y)).flatten(start_dim=1)
        return m._fc(m._dropout(y))

    def _stem(self, x, capture):
        m = self.qmodel
        keep = capture is not None
        x = x.contiguous(memory_format=torch.channels_last)
        first = self.blocks[0].first_consumer()
        if self.stem_affine is not None:
            z = m._conv_stem(x).contiguous(memory_format=torch.channels_last)
            codes = torch.empty((z.shape[0], z.shape[2], z.shape[3], first.cp_in),
                                dtype=first.code_dtype, device=x.device)
            y0 = torch.empty_like(z) if (keep or self.blocks[0].use_res) else None
            tq_ops._launch("act_encode_act", 4 * z.numel() + 2 * codes.numel(),
                           lambda: tq_native.act_encode_act(z, *first.quant, codes,
                                                            act="swish", out=y0,
                                                            affine=self.stem_affine))
        else:
            y0 = m._swish(m._bn0(m._conv_stem(x))).contiguous(
                memory_format=torch.channels_last)
            codes = torch.empty((y0.shape[0], y0.shape[2], y0.shape[3], first.cp_in),
                                dtype=first.code_dtype, device=x.device)
            tq_ops._launch("act_encode", 4 * y0.numel() + 2 * codes.numel(),
                           lambda: tq_native.act_encode(y0, True, *first.quant, codes))
        if keep:
            capture.append({"name": "stem", "kind": "stem", "out": y0, "codes_out": codes,
                            "quant": first.quant})
        return codes, y0

    def _body(self, codes, xin, y, capture=None):
        """The blocks and the head conv (into ``y``) as a generator: yields after each
        launch."""
        keep = capture is not None
        for i, b in enumerate(self.blocks):
            nxt = self.blocks[i + 1] if i + 1 < len(self.blocks) else None
            if b.expand is not None:
                # BN + swish + the dw conv's codes in the epilogue (the direct engine's swish
                # instantiation: 1x1 convs)
                h, hcodes, _ = b.expand(codes, out=True if keep else None, relu="swish",
                                        next_a=b.dw.consumer)
                yield
                if keep:
                    capture.append({"name": "block%d.expand" % i, "kind": "conv",
                                    "conv": b.expand, "codes_in": codes, "residual": None,
                                    "out": h, "codes_out": hcodes, "act": "swish"})
            else:
                hcodes = codes
            if b.has_se:
                d, _ = b.dw(hcodes, None, out=True, act="swish")
                yield
                g = b.gate(d)
                yield
                pcodes = torch.empty((d.shape[0], d.shape[2], d.shape[3], b.project.cp_in),
                                     dtype=b.project.code_dtype, device=d.device)
                tq_ops._launch("act_encode_act", 6 * d.numel(),
                               lambda: tq_native.act_encode_act(d, *b.project.quant, pcodes,
                                                                gate=g))
                yield
            else:
                d, pcodes = b.dw(hcodes, b.project, out=keep, act="swish")
                g = None
                yield
            if keep:
                capture.append({"name": "block%d.dw" % i, "kind": "dw", "conv": b.dw,
                                "codes_in": hcodes, "residual": None, "out": d,
                                "codes_out": pcodes, "act": "swish", "gate": g})
            consumer = nxt.first_consumer() if nxt is not None else self.head
            need_out = keep or (nxt is not None and nxt.use_res)
            xout, codes, _ = b.project(pcodes, out=True if need_out else None,
                                       residual=xin if b.use_res else None, relu=False,
                                       next_a=consumer)
            yield
            if keep:
                capture.append({"name": "block%d.project" % i, "kind": "conv",
                                "conv": b.project, "codes_in": pcodes,
                                "residual": xin if b.use_res else None, "out": xout,
                                "codes_out": codes, "act": None})
            xin = xout
        self.head(codes, out=y, relu=False)
        yield
        if keep:
            capture.append({"name": "head", "kind": "conv", "conv": self.head,
                            "codes_in": codes, "residual": None, "out": y, "codes_out": None,
                            "act": None})
