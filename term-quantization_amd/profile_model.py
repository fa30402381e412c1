"""Term-pair MAC and parameter-bit counting (the reference's profile_model.py:1-64).

The reference counts with a fork of pytorch-OpCounter (thop/), which does not import on
Python 3.10.  This module keeps the same public functions (``tr_conv2d_ops``,
``tr_linear_ops``, ``tr_lstm_ops``, ``get_model_ops``) and the same numbers: per-module fp32
``total_ops`` / ``total_params`` counters updated by forward hooks, summed in module order
in fp32 (thop/profile.py:59-128), so published values such as ResNet-18's 7,629,963,264
term-pair MACs at g=8, k=12, dt=3 come out bit-identical.
"""
import numpy as np
import torch
import torch.nn as nn

import tr_layer
from cnn_models.efficientnet import Conv2dStaticSamePadding


def _add(m, attr, value):
    # thop: m.total_ops += torch.Tensor([int(v)])  (fp32 buffer, fp32 add)
    setattr(m, attr, np.float32(getattr(m, attr)) + np.float32(int(value)))


def tr_conv2d_ops(m, x, y):
    """profile_model.py:8-26: out_elems * Cin/groups * kh*kw * min(dt, db) * (k_eff / g);
    counted only for groups == 1 and Cin > 3."""
    x = x[0]
    kernel_ops = torch.zeros(m.conv.weight.size()[2:]).numel()  # Kw x Kh
    total_ops = y.nelement() * (m.conv.in_channels // m.conv.groups * kernel_ops)
    if m.group_size == 1:
        weight_terms = min(m.num_terms, m.weight_bits)
    else:
        weight_terms = m.num_terms
    data_terms = min(m.data_terms, m.data_bits)
    alpha = weight_terms / m.group_size
    total_ops = data_terms * alpha * total_ops
    if x.shape[1] > 3 and m.conv.groups == 1:
        _add(m.conv, 'total_ops', int(total_ops))


def tr_linear_ops(m, x, y):
    """profile_model.py:28-46; parameter bits from compute_compressed_hese for g > 1."""
    x = x[0]
    total_ops = y.nelement() * m.linear.in_features
    if m.group_size == 1:
        weight_terms = min(m.num_terms, m.weight_bits)
    else:
        weight_terms = m.num_terms
    data_terms = min(m.data_terms, m.data_bits)
    alpha = weight_terms / m.group_size
    total_ops = data_terms * alpha * total_ops
    _add(m.linear, 'total_ops', int(total_ops))
    if m.group_size == 1:
        weight_bits = m.linear.weight.nelement() * m.weight_bits
    else:
        weight_bits = tr_layer.compute_compressed_hese(m.linear.weight, m.w_sf, m.weight_bits)
    _add(m.linear, 'total_params', int(weight_bits))


def tr_lstm_ops(m, x, y):
    x = x[0]


def zero_ops(m, x, y):
    _add(m, 'total_ops', 0)


def _count_relu(m, x, y):
    _add(m, 'total_ops', int(x[0].numel()))


def _count_bn(m, x, y):
    _add(m, 'total_ops', int(2 * x[0].numel()) if not m.training else 0)


def _count_convNd(m, x, y):
    kernel_ops = torch.zeros(m.weight.size()[2:]).numel()
    bias_ops = 1 if m.bias is not None else 0
    _add(m, 'total_ops', int(y.nelement() * (m.in_channels // m.groups * kernel_ops + bias_ops)))


def _count_avgpool(m, x, y):
    _add(m, 'total_ops', int(y.numel()))


def _count_upsample(m, x, y):
    per = {'linear': 5, 'bilinear': 11, 'bicubic': 259}.get(m.mode, 0)
    _add(m, 'total_ops', int(y.nelement() * per))


# thop's default table (thop/profile.py:20-55) for the module types that are not overridden
_DEFAULT_HOOKS = {
    nn.Conv1d: _count_convNd, nn.Conv3d: _count_convNd, nn.ConvTranspose1d: _count_convNd,
    nn.ConvTranspose2d: _count_convNd, nn.ConvTranspose3d: _count_convNd,
    nn.BatchNorm1d: _count_bn, nn.BatchNorm3d: _count_bn,
    nn.ReLU: zero_ops, nn.ReLU6: zero_ops, nn.LeakyReLU: _count_relu,
    nn.MaxPool1d: zero_ops, nn.MaxPool2d: zero_ops, nn.MaxPool3d: zero_ops,
    nn.AdaptiveMaxPool1d: zero_ops, nn.AdaptiveMaxPool2d: zero_ops,
    nn.AdaptiveMaxPool3d: zero_ops,
    nn.AvgPool1d: _count_avgpool, nn.AvgPool3d: _count_avgpool,
    nn.Dropout: zero_ops,
    nn.Upsample: _count_upsample, nn.UpsamplingBilinear2d: _count_upsample,
    nn.UpsamplingNearest2d: zero_ops,
}


def _profile(model, inputs, custom_ops):
    handles = []
    counted = []

    def eligible(m):
        return not (len(list(m.children())) > 0 and type(m) not in custom_ops)

    for m in model.modules():
        if not eligible(m):
            continue
        m.total_ops = np.float32(0)
        m.total_params = np.float32(0)
        counted.append(m)
        fn = custom_ops.get(type(m), _DEFAULT_HOOKS.get(type(m)))
        if fn is not None:
            handles.append(m.register_forward_hook(fn))

    training = model.training
    model.eval()
    try:
        with torch.no_grad():
            model(*inputs)
        total_ops = np.float32(0)
        total_params = np.float32(0)
        for m in model.modules():
            if eligible(m):
                total_ops = np.float32(total_ops + m.total_ops)
                total_params = np.float32(total_params + m.total_params)
    finally:
        model.train(training)
        for h in handles:
            h.remove()
        for m in counted:
            del m.total_ops
            del m.total_params
    return float(total_ops), float(total_params)


def get_model_ops(model, inputs):
    """(term-pair MACs, parameter bits) of one forward on ``inputs`` (profile_model.py:51-64)."""
    custom_ops = {
        tr_layer.TRConv2dLayer: tr_conv2d_ops,
        tr_layer.TRLinearLayer: tr_linear_ops,
        tr_layer.TRLSTMLayer: tr_lstm_ops,
        nn.Conv2d: zero_ops,
        Conv2dStaticSamePadding: zero_ops,
        nn.BatchNorm2d: zero_ops,
        nn.Linear: zero_ops,
        nn.AvgPool2d: zero_ops,
        nn.AdaptiveAvgPool2d: zero_ops,
    }
    return _profile(model, inputs, custom_ops)
