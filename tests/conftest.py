"""Test configuration.

Markers: ``gpu`` -- needs an MI355X (run with ``-m gpu`` on the GPU box); everything else
runs on the CPU-only build container.  The product package directory and the oracle are put
on sys.path; tests are the only product-side code allowed to import ``oracle``.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "term-quantization_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


# (cin, cout, k, stride, hin) of the 19 ResNet-18 TR convs
RESNET18_TR = [(64, 64, 3, 1, 56)] * 4 + [(64, 128, 3, 2, 56), (128, 128, 3, 1, 28),
                                          (64, 128, 1, 2, 56)] + \
    [(128, 128, 3, 1, 28)] * 2 + [(128, 256, 3, 2, 28), (256, 256, 3, 1, 14),
                                  (128, 256, 1, 2, 28)] + \
    [(256, 256, 3, 1, 14)] * 2 + [(256, 512, 3, 2, 14), (512, 512, 3, 1, 7),
                                  (256, 512, 1, 2, 14)] + [(512, 512, 3, 1, 7)] * 2


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
