"""The summation order of torch's fp32 CPU conv for the ResNet stem shape (CPU test).

DESIGN.md section 3 measures the fp32 spread of the stem against the correctly rounded
composition; its premise is that torch's CPU conv (and MIOpen's NHWC conv, checked on the GPU
by tests/test_gpu_fused_parity.py::test_stem_seam_within_the_fp32_spread: bit-identical on
all 51.4 M pooled values of the bench batch) is the sequential fp32 fma chain over (kernel
row, kernel column, input channel) -- one summation order, so MIOpen vs CPU measures order
identity, not the spread.  This pins the CPU half of that premise."""
import numpy as np
import torch
import torch.nn.functional as F


def _fmaf(a, b, c):
    # fp32 fma: the fp64 product of two fp32 values is exact; one rounding of the sum (the
    # double rounding through fp64 cannot matter at these magnitudes except on ties that
    # the check would report)
    return np.float32(np.float64(a) * np.float64(b) + np.float64(c))


def test_cpu_conv_is_the_row_column_channel_fma_chain():
    torch.manual_seed(0)
    x = torch.randn(1, 3, 24, 24)
    w = torch.empty(64, 3, 7, 7)
    torch.nn.init.kaiming_normal_(w, mode="fan_out", nonlinearity="relu")
    y = F.conv2d(x.contiguous(memory_format=torch.channels_last), w, None, 2, 3)
    xp = F.pad(x, (3, 3, 3, 3))[0].numpy()
    wn = w.numpy()
    exact = F.conv2d(x.double(), w.double(), None, 2, 3).float()
    same = differ_exact = 0
    for c in range(0, 64, 7):
        for ho in range(0, 12, 3):
            for wo in range(0, 12, 3):
                acc = np.float32(0)
                for ky in range(7):
                    for kx in range(7):
                        for ci in range(3):
                            acc = _fmaf(xp[ci, 2 * ho + ky, 2 * wo + kx], wn[c, ci, ky, kx], acc)
                same += int(acc == y[0, c, ho, wo].item())
                differ_exact += int(acc != exact[0, c, ho, wo].item())
    n = 10 * 4 * 4
    assert same == n, (same, n)
    # and that order is a genuinely different rounding from the correctly rounded conv
    assert differ_exact > n // 2, differ_exact
