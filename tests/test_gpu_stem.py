"""GPU parity of the fused ResNet stem (conv 7x7/2 on split-fp16 matrix cores + BN + ReLU +
max-pool + first-layer TR codes, tq_stem_conv_pool_encode) against an fp64 reference."""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import oracle
import tq_native
import tq_ops

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _bn_coefs(seed):
    torch.manual_seed(seed)
    bn = nn.BatchNorm2d(64).eval()
    with torch.no_grad():
        bn.weight.uniform_(-1.5, 1.5)  # negative scales: BN must come before the max
        bn.bias.uniform_(-0.3, 0.3)
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.5, 2.0)
    a = bn.weight.double() / torch.sqrt(bn.running_var.double() + bn.eps)
    return a.float().contiguous(), (bn.bias.double() - bn.running_mean.double() * a).float()


@pytest.mark.parametrize("n,h,w,fmt,xs", [(3, 32, 48, torch.float16, 2.0),
                                          (2, 224, 224, torch.float16, 2.0),
                                          (1, 64, 36, torch.int16, 2.0),
                                          (2, 20, 296, torch.float16, 2.0),
                                          (2, 32, 48, torch.float16, 1e-3),
                                          (2, 32, 48, torch.float16, 3e4),
                                          (1, 224, 224, torch.float16, 1e-30)])
def test_stem_conv_pool_matches_fp64(n, h, w, fmt, xs):
    """xs scales the N(0,1) input: the kernel's per-tile power-of-two input scaling keeps the
    fp16 split in range for inputs far from unit scale."""
    _stem_case(n, h, w, fmt, xs, h + w, (0.05, 9, 3))


@pytest.mark.parametrize("seed", range(16))
def test_stem_conv_pool_random_sweep(seed):
    """Seeded random stem shapes (H, W multiples of 4, W up to 448 -- one or two strips per
    wave, partial last tiles, narrow maps with idle waves), input scales 1e-4..1e4, code
    format and TR settings (sf, bit width 6-11, data terms 1-4)."""
    rng = np.random.default_rng(5000 + seed)
    h = 4 * int(rng.integers(2, 59))
    w = 4 * int(rng.integers(2, 113))
    fmt = torch.float16 if rng.random() < 0.7 else torch.int16
    xs = float(10.0 ** rng.uniform(-4, 4))
    quant = (float(10.0 ** rng.uniform(-2.5, -0.5)), int(rng.integers(6, 12)),
             int(rng.integers(1, 5)))
    _stem_case(int(rng.integers(1, 4)), h, w, fmt, xs, 5000 + seed, quant)


def _stem_case(n, h, w, fmt, xs, seed, quant):
    sf, bw, dt = quant
    torch.manual_seed(seed)
    x = (torch.randn(n, 3, h, w) * xs).contiguous(memory_format=torch.channels_last)
    wt = torch.empty(64, 3, 7, 7)
    nn.init.kaiming_normal_(wt, mode="fan_out", nonlinearity="relu")
    sc, sh = _bn_coefs(seed)
    ho, wo = h // 4, w // 4
    out = torch.full((n, 64, ho, wo), float("nan"), device=DEV).contiguous(
        memory_format=torch.channels_last)
    codes = torch.zeros((n, ho, wo, 64), dtype=fmt, device=DEV)
    wsplit = tq_ops.pack_stem_weight(wt.to(DEV))
    tq_native.stem_conv_pool_encode(x.to(DEV), wsplit, sc.to(DEV), sh.to(DEV), out,
                                    codes_a=codes, quant_a=(sf, bw, dt))
    got = out.cpu().double()
    # fp64 reference: conv -> BN (the fp32 coefficients) -> ReLU -> max-pool
    z = F.conv2d(x.double(), wt.double(), None, 2, 3)
    mag = F.conv2d(x.double().abs(), wt.double().abs(), None, 2, 3)
    sd, hd = sc.double().view(1, -1, 1, 1), sh.double().view(1, -1, 1, 1)
    ref = F.max_pool2d(torch.relu(z * sd + hd), 3, 2, 1)
    tol = 1e-5 * F.max_pool2d(mag * sd.abs() + hd.abs(), 3, 2, 1) + 1e-30
    err = (got - ref).abs()
    assert not torch.isnan(got).any()
    assert bool((err <= tol).all()), float((err / tol).max())
    # the codes are exactly TR of the fp32 output the kernel wrote (tr_layer.py:96-99)
    yq = oracle.tr(out.contiguous().cpu().numpy().reshape(1, -1, 1, 1), sf, bw, 1, dt)
    exp = np.rint(yq.reshape(out.shape) / np.float32(sf)).astype(np.int64)
    assert torch.equal(codes.cpu().long().permute(0, 3, 1, 2), torch.from_numpy(exp))


def test_stem_rejects_bad_shapes():
    x = torch.zeros((1, 3, 30, 32), device=DEV).contiguous(memory_format=torch.channels_last)
    out = torch.zeros((1, 64, 7, 8), device=DEV).contiguous(memory_format=torch.channels_last)
    wsplit = tq_ops.pack_stem_weight(torch.zeros(64, 3, 7, 7, device=DEV))
    sc = torch.ones(64, device=DEV)
    with pytest.raises(RuntimeError, match="H, W % 4"):
        tq_native.stem_conv_pool_encode(x, wsplit, sc, sc, out)


def test_stem_row_carry_is_bit_identical_to_separate_tiles():
    """One strip per wave (Wo <= 56): a workgroup walking several tiles down an image carries
    each tile's last conv row into the next tile instead of recomputing it -- only when both
    tiles scaled their inputs by the same power of two.  40 images (560 tiles: runs of 2-3
    tiles per workgroup, starting mid-image) with bands of rows scaled by 1e-3 / 40 (adjacent
    tiles with different scales) give the same bits as every image launched alone (14 tiles
    on 14 workgroups: no carry at all)."""
    torch.manual_seed(7)
    n = 40
    x = torch.randn(n, 3, 224, 224)
    x[:, :, 40:72] *= 1e-3    # tiles whose max |x| falls several binades
    x[:, :, 150:160] *= 40.0  # and one that rises
    x[1::3] *= 0.3
    x = x.contiguous(memory_format=torch.channels_last).to(DEV)
    wt = torch.empty(64, 3, 7, 7)
    nn.init.kaiming_normal_(wt, mode="fan_out", nonlinearity="relu")
    sc, sh = _bn_coefs(11)
    sc, sh = sc.to(DEV), sh.to(DEV)
    wsplit = tq_ops.pack_stem_weight(wt.to(DEV))

    def run(xb):
        out = torch.empty((xb.shape[0], 64, 56, 56), device=DEV).contiguous(
            memory_format=torch.channels_last)
        codes = torch.empty((xb.shape[0], 56, 56, 64), dtype=torch.float16, device=DEV)
        tq_native.stem_conv_pool_encode(xb, wsplit, sc, sh, out, codes_a=codes,
                                        quant_a=(0.05, 9, 3))
        return out, codes

    out, codes = run(x)
    for i in (0, 1, 2, 17, 39):
        o1, c1 = run(x[i:i + 1].contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
        assert torch.equal(out[i].view(torch.int32), o1[0].view(torch.int32)), i
        assert torch.equal(codes[i].view(torch.int16), c1[0].view(torch.int16)), i


def _exact_codes(x, wt, sc, sh, quant):
    """Codes of the correctly rounded stem: fp64 conv (exact products, fp64 sum) rounded once
    to fp32, BN as one fp32 fma (emulated in 80-bit long double: the product is exact, then
    a single rounding to fp32), ReLU, max-pool 3x3/2 pad 1, then oracle.tr.  Returns (fp32
    pooled values NCHW, integer codes NCHW)."""
    sf, bw, dt = quant
    z = F.conv2d(x.double(), wt.double(), None, 2, 3).float().numpy()
    ld = np.longdouble
    y = (z.astype(ld) * sc.detach().numpy().astype(ld).reshape(1, -1, 1, 1) +
         sh.detach().numpy().astype(ld).reshape(1, -1, 1, 1)).astype(np.float32)
    y = np.maximum(y, np.float32(0.0))
    pooled = F.max_pool2d(torch.from_numpy(y), 3, 2, 1).numpy()
    yq = oracle.tr(np.ascontiguousarray(pooled).reshape(1, -1, 1, 1), sf, bw, 1, dt)
    return pooled, np.rint(yq.reshape(pooled.shape) / np.float32(sf)).astype(np.int64)


def _exact_case(n, h, w, fmt, xs, seed, quant, scale_bands=False, workspace=None):
    sf, bw, dt = quant
    torch.manual_seed(seed)
    x = torch.randn(n, 3, h, w) * xs
    if scale_bands:  # tiles of very different max |x| (the error bound is per tile)
        x[:, :, h // 5:h // 3] *= 1e-3
        x[:, :, h // 2:h // 2 + 6] *= 30.0
    x = x.contiguous(memory_format=torch.channels_last)
    wt = torch.empty(64, 3, 7, 7)
    nn.init.kaiming_normal_(wt, mode="fan_out", nonlinearity="relu")
    sc, sh = _bn_coefs(seed)
    sc, sh = sc.detach(), sh.detach()
    ho, wo = h // 4, w // 4
    out = torch.full((n, 64, ho, wo), float("nan"), device=DEV).contiguous(
        memory_format=torch.channels_last)
    codes = torch.zeros((n, ho, wo, 64), dtype=fmt, device=DEV)
    wsplit = tq_ops.pack_stem_weight(wt.to(DEV))
    exact = tq_ops.pack_stem_exact(wt.to(DEV))
    tq_native.stem_conv_pool_encode(x.to(DEV), wsplit, sc.to(DEV), sh.to(DEV), out,
                                    codes_a=codes, quant_a=quant, exact=exact,
                                    workspace=workspace)
    codes_split = torch.zeros_like(codes)
    out_split = torch.empty_like(out)
    tq_native.stem_conv_pool_encode(x.to(DEV), wsplit, sc.to(DEV), sh.to(DEV), out_split,
                                    codes_a=codes_split, quant_a=quant)
    pooled, exp = _exact_codes(x, wt, sc, sh, quant)
    got = codes.cpu().long().permute(0, 3, 1, 2).numpy()
    split = codes_split.cpu().long().permute(0, 3, 1, 2).numpy()
    # every code is the correctly rounded conv's code
    assert np.array_equal(got, exp), int((got != exp).sum())
    # and still TR of the fp32 output the kernels wrote (the fix-up rewrites both)
    yq = oracle.tr(out.contiguous().cpu().numpy().reshape(1, -1, 1, 1), sf, bw, 1, dt)
    assert np.array_equal(np.rint(yq.reshape(out.shape) / np.float32(sf)).astype(np.int64), got)
    # outputs the fix-up did not touch are the split kernel's bits; the others the exact value
    o = out.cpu().numpy()
    os_ = out_split.cpu().numpy()
    touched = o.view(np.int32) != os_.view(np.int32)
    assert np.array_equal(o[touched], pooled[touched])
    return int((split != exp).sum()), int(touched.sum()), got.size


@pytest.mark.parametrize("n,h,w,fmt,xs,bands", [(2, 224, 224, torch.float16, 1.0, False),
                                                (3, 32, 48, torch.int16, 2.0, False),
                                                (2, 20, 296, torch.float16, 3e3, False),
                                                (4, 224, 224, torch.float16, 1.0, True),
                                                (1, 64, 36, torch.float16, 1e-3, True)])
def test_stem_exact_fixup_gives_the_correctly_rounded_codes(n, h, w, fmt, xs, bands):
    """The exact fix-up (tq_ops.pack_stem_exact): every code equals the code of the correctly
    rounded fp32 conv -> the same BN fma -> ReLU -> max-pool, on shapes where the split-fp16
    result alone flips codes.  sf is small (0.002: 9-bit codes span ~1, so many quotients sit
    near midpoints) to exercise the fix-up heavily."""
    flips_split, touched, total = _exact_case(n, h, w, fmt, xs, 900 + h + w, (0.002, 9, 3),
                                              bands)
    print("exact stem %dx%dx%d: split-only flips %d, fixed-up outputs %d of %d"
          % (n, h, w, flips_split, touched, total))


@pytest.mark.parametrize("seed", range(8))
def test_stem_exact_fixup_random_sweep(seed):
    """Seeded random shapes, input scales and TR settings for the exact fix-up."""
    rng = np.random.default_rng(7000 + seed)
    h = 4 * int(rng.integers(2, 59))
    w = 4 * int(rng.integers(2, 113))
    fmt = torch.float16 if rng.random() < 0.7 else torch.int16
    xs = float(10.0 ** rng.uniform(-3, 3))
    quant = (float(10.0 ** rng.uniform(-3, -1)) * xs, int(rng.integers(6, 12)),
             int(rng.integers(1, 5)))
    _exact_case(int(rng.integers(1, 4)), h, w, fmt, xs, 7000 + seed, quant,
                bool(rng.random() < 0.5))


@pytest.mark.parametrize("fmt", [torch.float16, torch.int16])
def test_stem_exact_fixup_large_quotients(fmt):
    """11-bit codes with quotients up to ~2000 (sf 0.0015 on N(0, 1) inputs): the listing's
    rounding slack grows with the quotient (2^-21 r + 2^-23 max|shift| / sf), where a flat
    slack stops covering the fp32 rounding terms (r above ~600).  Every code is the correctly
    rounded conv's."""
    flips_split, touched, total = _exact_case(6, 224, 224, fmt, 1.0, 4711, (0.0015, 11, 3))
    print("large quotients: split-only flips %d, fixed-up outputs %d of %d"
          % (flips_split, touched, total))


def test_stem_exact_fixup_long_segments():
    """Workgroup segments longer than the fix-up's LDS entry stage (4096 entries; the rest are
    read from the workspace in global memory): 300 images of 16 x 336 (300 tiles over <= 256
    workgroups, so some take two tiles of 4 x 84 pool pixels x 16 channel quads), and an sf
    / bitwidth at which the error bound covers a large part of every quotient's unit interval
    (most quads listed).  Every code is still the correctly rounded conv's."""
    n, h, w = 300, 16, 336
    ws = tq_native.stem_workspace(n, h, w, DEV).zero_()  # (counts past the grid stay 0)
    _, touched, total = _exact_case(n, h, w, torch.int16, 1.0, 4242, (1e-4, 14, 3),
                                    workspace=ws)
    counts = ws[:4096].view(torch.int32).cpu().numpy()
    assert counts.max() > 4096, int(counts.max())
    print("long segments: max %d entries per workgroup, %d listed in all, %d outputs changed "
          "of %d" % (int(counts.max()), int(counts.sum()), touched, total))


def test_stem_exact_rejects_partial_args():
    x = torch.zeros((1, 3, 32, 32), device=DEV).contiguous(memory_format=torch.channels_last)
    out = torch.zeros((1, 64, 8, 8), device=DEV).contiguous(memory_format=torch.channels_last)
    wt = torch.zeros(64, 3, 7, 7, device=DEV)
    wsplit = tq_ops.pack_stem_weight(wt)
    w64, wb = tq_ops.pack_stem_exact(wt)
    sc = torch.ones(64, device=DEV)
    small = torch.empty(16, dtype=torch.uint8, device=DEV)
    with pytest.raises(RuntimeError, match="workspace too small"):
        tq_native.stem_conv_pool_encode(x, wsplit, sc, sc, out, exact=(w64, wb),
                                        workspace=small)
