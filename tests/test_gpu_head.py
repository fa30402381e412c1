"""The fused ResNet executor's classifier head (tq_avgpool_fc_f32: avgpool -> flatten -> fc,
fp32 torch in the reference, torchvision ResNet.forward) against an fp64 composition."""
import pytest
import torch

import tq_native

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("n,c,h,w,o", [(256, 512, 7, 7, 1000), (3, 64, 5, 5, 10),
                                       (2, 300, 1, 1, 7), (17, 4, 3, 2, 33)])
def test_avgpool_fc_matches_fp64(n, c, h, w, o):
    torch.manual_seed(n + c + o)
    x = torch.relu(torch.randn(n, c, h, w)).contiguous(memory_format=torch.channels_last)
    wt = torch.randn(o, c) * 0.05
    b = torch.randn(o) * 0.1
    got = tq_native.avgpool_fc(x.to(DEV), wt.to(DEV), b.to(DEV)).cpu().double()
    p = x.double().mean(dim=(2, 3))
    ref = p @ wt.double().t() + b.double()
    mag = p.abs() @ wt.double().abs().t() + b.double().abs()
    assert bool(((got - ref).abs() <= 1e-5 * mag + 1e-30).all())
    got0 = tq_native.avgpool_fc(x.to(DEV), wt.to(DEV), None).cpu().double()
    assert bool(((got0 - (ref - b.double())).abs() <= 1e-5 * mag + 1e-30).all())


def test_avgpool_fc_rejects_nchw():
    x = torch.zeros(2, 8, 3, 3, device=DEV)
    with pytest.raises(RuntimeError, match="channels_last"):
        tq_native.avgpool_fc(x, torch.zeros(4, 8, device=DEV), None)
