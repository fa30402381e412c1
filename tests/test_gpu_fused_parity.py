"""Teacher-forced parity of the measured path: the fused ResNet-18 executor (tq_fuse.py) that
bench.py times, at the bench config (BASELINE configs[1]: g=8, k=12, wb=db=9, dt=3, batch
256 x 3 x 224 x 224, bench.py's calibration), checked conv by conv against the oracle.

For every one of the 19 term-pair convs, on a sample of the batch's images:
  (i)  its input codes are bit-exact oracle.tr() of the fp32 tensor they encode
       (tr_layer.py:96-99: the producing epilogue's stored output, or the stem's), and the
       channel padding holds zero codes;
  (ii) its fp32 output is within 1e-5 of the fp64 composition conv -> BN -> (+ identity)
       -> ReLU of those same codes (tr_layer.py:124-126 plus the torchvision block), with
       the identity the kernel was handed.
The capture mode only adds fp32 stores; the bench-mode logits must be bit-identical to it.

A second test runs the module path (TRConv2dLayer + torch BN/ReLU/add, the reference
composition) teacher-forced on the fused path's inputs: every activation-code mismatch
between the two must be a one-step flip of the quantized integer whose two fp32 values sit
within a few ulps of each other -- i.e. a rounding-midpoint straddle caused by the BN-fold
rounding, never an indexing or epilogue bug."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import oracle
import tq_fuse

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SAMPLE = [0, 131, 255]


def _out(t, idx):
    """Sample images of an fp32 [N, C, H, W] (channels_last) tensor, as fp64 NCHW."""
    return t[idx].double().cpu().contiguous()


def _codes(t, idx, c):
    """Sample images of an NHWC [N, H, W, Cp] code tensor, first c channels, fp64 NCHW."""
    return t[idx][..., :c].double().permute(0, 3, 1, 2).cpu().contiguous()


def _tr_codes(y, quant):
    """Integer term sums oracle.tr would produce for fp32 y (NCHW fp64 holding fp32 values)."""
    sf, db, dt = quant
    yq = oracle.tr(y.float().numpy().reshape(1, -1, 1, 1), sf, db, 1, dt).reshape(y.shape)
    return np.rint(yq.astype(np.float64) / float(np.float32(sf))).astype(np.int64)


def _reference(conv, codes_in, residual, idx, relu=True):
    """fp64 conv -> BN -> (+residual) -> ReLU of the sampled input codes (teacher forced);
    the downsample branch is conv -> BN only."""
    layer = conv.layer
    c = layer.conv
    cin = c.in_channels
    sf_x = float(np.float32(conv.quant[0]))
    xq = _codes(codes_in, idx, cin) * sf_x
    wq = c.weight.detach().double().cpu()  # TR(w) = v_w * sf_w exactly (fp32)
    z = F.conv2d(xq, wq, None, c.stride, c.padding, c.dilation)
    mag = F.conv2d(xq.abs(), wq.abs(), None, c.stride, c.padding, c.dilation)
    if c.bias is not None:
        z = z + c.bias.detach().double().cpu().view(1, -1, 1, 1)
    bn = conv.bn
    a = (bn.weight.detach().double() / torch.sqrt(bn.running_var.double() + bn.eps)).cpu()
    y = (z - bn.running_mean.double().cpu().view(1, -1, 1, 1)) * a.view(1, -1, 1, 1) + \
        bn.bias.detach().double().cpu().view(1, -1, 1, 1)
    res = torch.zeros_like(y)
    if residual is not None:
        res = _out(residual, idx)
        y = y + res
    if relu:
        y = torch.relu(y)
    bound = 1e-5 * (torch.maximum(y.abs(), mag * a.abs().view(1, -1, 1, 1)) + res.abs()) + 1e-30
    return y, bound


def _check_input_codes(rec, src, idx):
    conv = rec["conv"]
    cin = conv.layer.conv.in_channels
    got = rec["codes_in"][idx].long().cpu()
    exp = _tr_codes(_out(src, idx), conv.quant)
    assert torch.equal(got[..., :cin].permute(0, 3, 1, 2), torch.from_numpy(exp)), rec["name"]
    if got.shape[-1] > cin:
        assert not got[..., cin:].any(), rec["name"] + ": pad channels"


@pytest.fixture(scope="module")
def bench_model():
    import os
    import bench
    old = os.environ.get("TQ_CONV_ENGINE")
    os.environ["TQ_CONV_ENGINE"] = "mfma"
    try:
        dev = torch.device(DEV)
        _, qmodel, _ = bench.build_model(dev, 256, 0)   # bench.py's model + calibration
    finally:
        if old is None:
            os.environ.pop("TQ_CONV_ENGINE")
        else:
            os.environ["TQ_CONV_ENGINE"] = old
    import util
    x, _ = util.SyntheticImageNet(512, 256, seed=0, device=dev).batch(0)  # bench batch 0
    return qmodel, x.contiguous(memory_format=torch.channels_last)


def test_fused_executor_teacher_forced_at_bench_config(bench_model):
    qmodel, x = bench_model
    fused = tq_fuse.FusedResNet(qmodel)
    assert fused.stem_w is not None  # the fused stem kernel, as in the bench
    with torch.no_grad():
        logits = fused(x)
        rec = []
        logits_cap = fused(x, capture=rec)
    torch.cuda.synchronize()
    assert torch.equal(logits, logits_cap)  # capture adds stores only
    convs = [r for r in rec if r["name"] != "stem"]
    assert len(convs) == 19
    idx = SAMPLE
    block_out = rec[0]["out"]  # fp32 tensor the next conv1 / downsample codes encode
    conv1_out = None
    for r in convs:
        conv = r["conv"]
        if r["name"].endswith("conv2"):
            src = conv1_out
        else:
            src = block_out
        _check_input_codes(r, src, idx)
        y_ref, bound = _reference(conv, r["codes_in"], r["residual"], idx,
                                  relu=not r["name"].endswith("downsample"))
        y = _out(r["out"], idx)
        err = (y - y_ref).abs()
        assert bool((err <= bound).all()), "%s: max err / bound %.3g" % (
            r["name"], float((err / bound).max()))
        if r["name"].endswith("conv1"):
            conv1_out = r["out"]
        elif r["name"].endswith("conv2"):
            block_out = r["out"]


@pytest.mark.parametrize("nstreams", [2, 4])
def test_stream_split_is_bit_identical(bench_model, nstreams):
    """forward_streams (bench.py --streams): the batch in image chunks on concurrent HIP
    streams gives exactly forward()'s logits."""
    qmodel, x = bench_model
    fused = tq_fuse.FusedResNet(qmodel)
    streams = [torch.cuda.Stream(DEV) for _ in range(nstreams)]
    with torch.no_grad():
        ref = fused(x)
        for _ in range(2):
            got = fused.forward_streams(x, streams)
    torch.cuda.synchronize()
    assert torch.equal(ref, got)


def _quantize(y, quant):
    """q of kernels/tr_cuda_kernel.cu:21-23 for fp32 values y >= 0 (numpy)."""
    sf, db, _ = quant
    r = (np.abs(y.astype(np.float32)) / np.float32(sf)).astype(np.float32)
    t = r.astype(np.float64) + 0.5
    return np.minimum(np.floor(t), 2.0 ** db - 1).astype(np.int64)


def test_module_path_teacher_forced_code_flips_are_midpoint_straddles(bench_model):
    """The module path (reference composition: TRConv2dLayer forward, torch BN, ReLU, add)
    and the fused executor fed the same inputs, layer by layer, on 8 images."""
    qmodel, x = bench_model
    x = x[:8].contiguous(memory_format=torch.channels_last)
    fused = tq_fuse.FusedResNet(qmodel)
    with torch.no_grad():
        rec = []
        fused(x, capture=rec)
        # stem: module path = MIOpen conv + torch BN/ReLU/max-pool
        m = qmodel
        stem_mod = m.maxpool(m.relu(m.bn1(m.conv1(x))))
        stem_fused = rec[0]["out"]
        # (near-fp32 split-fp16 conv vs MIOpen fp32: both within ~1e-6 of fp64 relative to
        # the products' magnitude; test_gpu_stem.py holds the per-element fp64 bound)
        d = (stem_mod - stem_fused).abs().max().item()
        assert d <= 1e-5 * stem_mod.abs().max().item(), d
        # the per-block modules of the converted model, in executor order
        blocks = [b for layer in (m.layer1, m.layer2, m.layer3, m.layer4) for b in layer]
        convs = [r for r in rec if r["name"] != "stem"]
        it = iter(convs)
        block_in = stem_fused
        flips = total = 0
        for blk in blocks:
            r1 = next(it)
            y1_mod = blk.relu(blk.bn1(blk.conv1(block_in)))
            pairs = [(r1, y1_mod, r1["out"], fused_next(rec, r1))]
            if blk.downsample is not None:
                rd = next(it)
                identity = blk.downsample(block_in)
                d = (identity - rd["out"]).abs().max().item()
                assert d <= 1e-5 * (rd["out"].abs().max().item() + 1e-30), rd["name"]
            r2 = next(it)
            # teacher forced: conv2 sees the fused path's conv1 output and identity
            y2_mod = blk.relu(blk.bn2(blk.conv2(r1["out"])) + r2["residual"])
            pairs.append((r2, y2_mod, r2["out"], fused_next(rec, r2)))
            for r, ym, yf, (codes, quant) in pairs:
                ym = ym.contiguous(memory_format=torch.channels_last)
                scale = yf.abs().amax().item() + 1e-30
                assert (ym - yf).abs().max().item() <= 1e-5 * scale, r["name"]
                if codes is None:
                    continue
                c = yf.shape[1]
                got = codes[..., :c].long().cpu().permute(0, 3, 1, 2).numpy()
                ymn = ym.float().cpu().numpy()
                yfn = yf.float().cpu().numpy()
                exp_mod = _tr_codes(torch.from_numpy(ymn).double(), quant)
                assert np.array_equal(got, _tr_codes(torch.from_numpy(yfn).double(), quant))
                mism = got != exp_mod
                total += got.size
                if not mism.any():
                    continue
                flips += int(mism.sum())
                qm, qf = _quantize(ymn[mism], quant), _quantize(yfn[mism], quant)
                assert np.all(np.abs(qm - qf) == 1), r["name"]
                lo = np.minimum(qm, qf).astype(np.float64) + 0.5  # the straddled midpoint
                sf = float(np.float32(quant[0]))
                for v in (ymn[mism], yfn[mism]):
                    ulp = np.spacing(np.abs(v).astype(np.float32)).astype(np.float64)
                    assert np.all(np.abs(v.astype(np.float64) - lo * sf) <= 8 * ulp + lo * sf *
                                  2.0 ** -22), r["name"]
            block_in = r2["out"]
        print("BN-fold seam: %d of %d activation codes (module path vs fused executor, teacher "
              "forced, 8 images) differ (%.2e), all one-step midpoint straddles"
              % (flips, total, flips / max(total, 1)))
        assert total > 0 and flips <= total * 1e-4, (flips, total)


def test_free_running_drift_from_module_path(bench_model):
    """The measured path free-running: FusedResNet (what bench.py times) against the module
    path (TRConv2dLayer + torch BN / ReLU / add: the reference composition) on the whole
    256-image bench batch, with nothing teacher forced -- so the midpoint code flips of the
    stem and BN-fold seams propagate through all 19 layers.  Records the top-1 agreement and
    the logit deviation max |dlogit| / max |logit| (measured 1.0000 and
    4.9e-3, bounded at about twice that)."""
    qmodel, x = bench_model
    fused = tq_fuse.FusedResNet(qmodel)
    with torch.no_grad():
        lf = fused(x).double()
        lm = qmodel(x).double()
    torch.cuda.synchronize()
    agree = float((lf.argmax(1) == lm.argmax(1)).double().mean())
    dev = float((lf - lm).abs().max() / lm.abs().max())
    mean_dev = float((lf - lm).abs().mean() / lm.abs().mean())
    print("free-running drift (256 images): top-1 agreement %.4f, max |dlogit| / max |logit| "
          "%.3e, mean |dlogit| / mean |logit| %.3e" % (agree, dev, mean_dev))
    assert agree >= 0.99 and dev <= 1e-2, (agree, dev)


def fused_next(rec, r):
    """(codes the fused conv emitted for its next consumer, that consumer's quantizer)."""
    names = [q["name"] for q in rec]
    i = names.index(r["name"])
    for q in rec[i + 1:]:
        if "conv" in q and q["codes_in"] is r["codes_a"]:
            return r["codes_a"], q["conv"].quant
    return None, None


def test_calibration_matches_the_reference_fp32_loop(bench_model):
    """Seam 1, calibration: the literal loop of tr_layer.py:43-54 -- 2048 HIP tr() calls and
    torch's fp32 (hist * (x - xh)**2).sum() on the GPU, then the first arg-min -- on the 19
    bench histograms, against the sf tq_mse_profile chose (fp64 sums of the same fp32 per-bin
    terms).  Where the two differ, the flip must be explained by the reference's own fp32
    reduction: the exact error gap between the two candidates is no larger than the rounding
    of the reference's two fp32 sums."""
    import tr_layer
    qmodel, _ = bench_model
    layers = [m for m in qmodel.modules() if isinstance(m, tr_layer.TRConv2dLayer)]
    assert len(layers) == 19
    differ = []
    for li, m in enumerate(layers):
        q = m.input_quant
        hist = q.hist_bins
        x = torch.linspace(q.minv, q.maxv, len(hist)).to(DEV)
        sfs = torch.linspace(1e-8, q.maxv, 2048).tolist()
        errs32, errs64 = [], []
        for sf in sfs:
            xh = tr_layer.tr_cuda.tr(x.view(-1, 1, 1, 1), sf, q.data_bits, 1,
                                     q.data_terms).view(-1)
            t = hist * (x - xh) ** 2
            errs32.append(t.sum())
            errs64.append(t.double().sum())
        e32 = torch.stack(errs32).cpu()
        e64 = torch.stack(errs64).cpu()
        i_ref = int(torch.argmin(e32).item())
        sf_ref = sfs[i_ref]
        i_got = sfs.index(q.sf)
        if i_got != i_ref:
            gap = float(e64[i_ref] - e64[i_got])
            rnd = abs(float(e32[i_ref]) - float(e64[i_ref])) + \
                abs(float(e32[i_got]) - float(e64[i_got]))
            assert 0.0 <= gap <= rnd, (li, i_ref, i_got, gap, rnd)
            differ.append((li, i_ref, i_got, gap, rnd))
        else:
            assert q.sf == sf_ref
    print("calibration seam: %d of 19 bench layers pick a different sf than the reference's "
          "fp32 loop %s" % (len(differ), differ))


def _exact_stem(m, x):
    """The correctly rounded stem composition on the GPU: conv1 in fp64 (exact products, fp64
    sums) rounded once to fp32, bn1 as the executor's fp32 affine (scale, shift) emulated in
    fp64 (exact product, one more rounding), ReLU, max-pool -- NHWC fp32."""
    bn = m.bn1
    a = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
    sc = a.float().double().view(1, -1, 1, 1)
    sh = (bn.bias.detach().double() - bn.running_mean.detach().double() * a).float().double()
    out = []
    for xc in x.split(32):
        z = F.conv2d(xc.double(), m.conv1.weight.detach().double(), None, 2, 3).float()
        y = torch.relu((z.double() * sc + sh.view(1, -1, 1, 1)).float())
        out.append(F.max_pool2d(y, 3, 2, 1).permute(0, 2, 3, 1).contiguous().cpu())
    return torch.cat(out).numpy()


def test_fused_stem_codes_are_the_correctly_rounded_stems(bench_model):
    """Seam 2, the stem, on the whole 256-image bench batch: layer1.0's input codes from the
    exact fused stem (split-fp16 MFMA conv + the exact fix-up of every output within the
    split's error bound of a rounding midpoint) equal oracle.tr() of the correctly
    rounded composition -- fp64 conv rounded once to fp32, the same BN fma, ReLU, max-pool --
    at every one of the 51,380,224 codes.  Prints how many the split stem alone flips."""
    qmodel, x = bench_model
    fused = tq_fuse.FusedResNet(qmodel, stem="exact")
    assert fused.stem_w is not None and fused.stem_exact is not None
    with torch.no_grad():
        rec = []
        fused(x, capture=rec)
        rec_s = []
        tq_fuse.FusedResNet(qmodel, stem="fused")(x, capture=rec_s)
        truth = _exact_stem(qmodel, x)
    quant = rec[1]["conv"].quant
    got = rec[1]["codes_in"][..., :64].float().cpu().numpy().astype(np.int64)
    split = rec_s[1]["codes_in"][..., :64].float().cpu().numpy().astype(np.int64)
    exp = _tr_ints(truth, quant)
    flips, flips_split = int((got != exp).sum()), int((split != exp).sum())
    print("stem seam (256 images, %d codes): fused exact stem vs correctly rounded %d; "
          "split-fp16 stem alone %d" % (got.size, flips, flips_split))
    assert flips == 0, flips


def _tr_ints(y, quant):
    """oracle.tr integer term sums of an NHWC fp32 array (threaded over 8 chunks)."""
    from concurrent.futures import ThreadPoolExecutor
    sf, db, dt = quant
    flat = y.reshape(-1)
    out = np.empty_like(flat)
    bounds = np.linspace(0, flat.size, 17).astype(np.int64)

    def run(j):
        lo, hi = bounds[j], bounds[j + 1]
        out[lo:hi] = oracle.tr(flat[lo:hi].reshape(1, -1, 1, 1), sf, db, 1, dt).reshape(-1)
    with ThreadPoolExecutor(8) as ex:
        list(ex.map(run, range(16)))
    return np.rint(out.astype(np.float64) / float(np.float32(sf))).astype(np.int64).reshape(
        y.shape)


def _gemm_order_stem(m, x):
    """The reference composition with the stem conv as an fp32 im2col GEMM (unfold + rocBLAS
    sgemm: K in (channel, row, column) order, blocked sums -- the data layout and summation
    order of an NCHW implicit-GEMM conv such as the reference's cuDNN one), then torch's bn1,
    ReLU and max-pool.  NHWC fp32."""
    w = m.conv1.weight.detach().reshape(64, -1)
    out = []
    for xc in x.detach().split(32):
        n, _, h, wd = xc.shape
        cols = F.unfold(xc.contiguous(), 7, padding=3, stride=2)          # [n, 147, L]
        z = torch.matmul(w, cols).view(n, 64, h // 2, wd // 2)
        with torch.no_grad():
            out.append(m.maxpool(m.relu(m.bn1(z))).permute(0, 2, 3, 1).contiguous().cpu())
    return torch.cat(out).numpy()


def test_stem_seam_within_the_fp32_spread(bench_model):
    """Is the fused stem inside the spread of fp32 stems?  On the whole 256-image bench
    batch, layer1.0's input codes as TR of (a) MIOpen's fp32 conv1 -> bn1 -> relu -> maxpool
    (the module path on the GPU, the reference composition), (b) the same composition in
    fp32 on the CPU, (e) the same with conv1 as an fp32 im2col GEMM (another summation
    order: (channel, row, column) K order, blocked sums), (c) the fused stem (split-fp16
    conv, the bench's default), (x) the exact fused stem (+ the fix-up: the correctly rounded
    conv's codes, t), and (d) the executor's --stem fp32 leg (MIOpen conv + the
    BN/ReLU/max-pool/codes kernel).

    (a) and (b) turn out to be one summation order -- torch's CPU conv and MIOpen's NHWC fp32
    conv are both the sequential fma chain over (row, column, channel), bit for bit the same
    values (printed) -- so their 0 flips measure order identity, not the fp32 spread; the
    spread is what a different fp32 order gives, (a) vs (e).  Every pair's flips must be
    one-step midpoint straddles.  The fused stem may flip no more codes against the
    correctly rounded stem than either fp32 order does (it is at least as accurate as the
    reference's fp32 conv), and the exact stem no more against (a) or (b) than the two fp32
    orders flip between themselves.  Prints the counts."""
    qmodel, x = bench_model
    m = qmodel
    with torch.no_grad():
        rec = []
        tq_fuse.FusedResNet(qmodel, stem="fused")(x, capture=rec)
        recx = []
        tq_fuse.FusedResNet(qmodel, stem="exact")(x, capture=recx)
        rec32 = []
        tq_fuse.FusedResNet(qmodel, stem="fp32")(x, capture=rec32)
        yt = _exact_stem(m, x)
        ya = m.maxpool(m.relu(m.bn1(m.conv1(x))))
        ye = _gemm_order_stem(m, x)
        import copy
        c1, b1 = copy.deepcopy(m.conv1).cpu(), copy.deepcopy(m.bn1).cpu()
        yb = m.maxpool(m.relu(b1(c1(x.cpu().contiguous()))))
    quant = rec[1]["conv"].quant
    nhwc = lambda t: t.permute(0, 2, 3, 1).contiguous().cpu().numpy()  # noqa: E731
    ya, yb = nhwc(ya), nhwc(yb)
    qa, qb, qe = _tr_ints(ya, quant), _tr_ints(yb, quant), _tr_ints(ye, quant)
    qt = _tr_ints(yt, quant)
    qc = rec[1]["codes_in"][..., :64].float().cpu().numpy().astype(np.int64)
    qx = recx[1]["codes_in"][..., :64].float().cpu().numpy().astype(np.int64)
    qd = rec32[1]["codes_in"][..., :64].float().cpu().numpy().astype(np.int64)
    vals = {"a": ya, "b": yb, "c": nhwc(rec[0]["out"]), "d": nhwc(rec32[0]["out"]), "e": ye,
            "x": nhwc(recx[0]["out"]), "t": yt}
    codes = {"a": qa, "b": qb, "c": qc, "d": qd, "e": qe, "x": qx, "t": qt}
    flips = {}
    for p, q in (("a", "b"), ("a", "e"), ("b", "e"), ("c", "a"), ("c", "b"), ("c", "e"),
                 ("d", "a"), ("d", "b"), ("c", "d"), ("x", "a"), ("x", "b"), ("a", "t"),
                 ("e", "t"), ("c", "t"), ("x", "t")):
        mism = codes[p] != codes[q]
        flips[p + q] = int(mism.sum())
        if flips[p + q]:
            qp, qq = _quantize(vals[p][mism], quant), _quantize(vals[q][mism], quant)
            assert np.all(np.abs(qp - qq) == 1), p + q
            mid = np.minimum(qp, qq).astype(np.float64) + 0.5
            s32 = np.float32(quant[0])
            rp = (np.abs(vals[p][mism]) / s32).astype(np.float32).astype(np.float64)
            rq = (np.abs(vals[q][mism]) / s32).astype(np.float32).astype(np.float64)
            assert np.all((np.minimum(rp, rq) <= mid) & (mid <= np.maximum(rp, rq))), p + q
    total = qa.size
    bits_ab = int((ya.view(np.int32) != yb.view(np.int32)).sum())
    bits_ae = int((ya.view(np.int32) != ye.view(np.int32)).sum())
    print("stem fp32 spread (%d images, %d codes): pooled fp32 values differing bitwise: MIOpen "
          "vs CPU %d, MIOpen vs im2col GEMM %d; code flips: MIOpen vs CPU %d, MIOpen vs GEMM %d, "
          "CPU vs GEMM %d; against the correctly rounded stem: MIOpen %d, GEMM %d, fused stem "
          "%d, exact stem %d; fused stem vs MIOpen %d, vs CPU %d, vs GEMM %d; exact stem vs "
          "MIOpen %d, vs CPU %d; --stem fp32 leg vs MIOpen %d, vs CPU %d; fused vs fp32 leg %d"
          % (x.shape[0], total, bits_ab, bits_ae, flips["ab"], flips["ae"], flips["be"],
             flips["at"], flips["et"], flips["ct"], flips["xt"], flips["ca"], flips["cb"],
             flips["ce"], flips["xa"], flips["xb"], flips["da"], flips["db"], flips["cd"]))
    assert flips["xt"] == 0, flips
    assert flips["ct"] <= min(flips["at"], flips["et"]), flips
    spread = max(flips["ab"], flips["ae"], flips["be"])
    assert flips["xa"] <= spread and flips["xb"] <= spread, flips
