"""CNN model zoo and TR conversion -- the reference's cnn_models package
(cnn_models/__init__.py:1-70) with the same functions and layer-selection rules.

The architectures are defined in this package (torchvision / efficientnet_pytorch are not
installed and there is no network for pretrained downloads).  ``pretrained=True`` loads a
local state_dict from ``$TQ_PRETRAINED_DIR/<arch>.pth`` (weights only) and raises if there
is none; ``pretrained=False`` gives the architecture's default random initialisation.
"""
import os
from copy import deepcopy

import torch
import torch.nn as nn

from tr_layer import TRConv2dLayer
from cnn_models.efficientnet import Conv2dStaticSamePadding, EfficientNet, efficientnet_b0_model
from cnn_models.mobilenet import mobilenet_v2 as _mobilenet_v2
from cnn_models.resnet import resnet18 as _resnet18
from cnn_models.vgg import alexnet as _alexnet, vgg16_bn as _vgg16_bn


def model_names():
    return ['alexnet', 'vgg16_bn', 'resnet18', 'efficientnet_b0', 'mobilenet_v2']


def _load_pretrained(model, arch):
    root = os.environ.get('TQ_PRETRAINED_DIR', '')
    path = os.path.join(root, arch + '.pth')
    if not root or not os.path.exists(path):
        raise RuntimeError(
            "pretrained=True needs a local state_dict at $TQ_PRETRAINED_DIR/%s.pth (no network "
            "access); use pretrained=False / --synthetic for random weights" % arch)
    model.load_state_dict(torch.load(path, map_location='cpu', weights_only=True))
    return model


def _build(arch, ctor, pretrained):
    model = ctor()
    return _load_pretrained(model, arch) if pretrained else model


def alexnet(pretrained=True):
    return _build('alexnet', _alexnet, pretrained)


def vgg16_bn(pretrained=True):
    return _build('vgg16_bn', _vgg16_bn, pretrained)


def resnet18(pretrained=True):
    return _build('resnet18', _resnet18, pretrained)


def mobilenet_v2(pretrained=True):
    return _build('mobilenet_v2', _mobilenet_v2, pretrained)


def efficientnet_b0(pretrained=True):
    # cnn_models/__init__.py:21-25 (EfficientNet.from_pretrained / from_name)
    return _build('efficientnet_b0', efficientnet_b0_model, pretrained)


def is_conv_layer(layer):
    return isinstance(layer, (nn.Conv2d, Conv2dStaticSamePadding))


def replace_conv_layers(model, tr_params, data_bits, data_terms):
    """Swap every conv except the first for a TRConv2dLayer (cnn_models/__init__.py:30-50)."""
    curr_layer = 0
    for name, layer in list(model.named_modules()):
        if is_conv_layer(layer):
            if curr_layer == 0:
                curr_layer += 1
                continue

            module_keys = name.split('.')
            module = model
            for k in module_keys[:-1]:
                module = module._modules[k]

            weight_bits, group_size, weight_terms = tr_params[curr_layer]
            layer = TRConv2dLayer(layer, data_bits, data_terms, weight_bits,
                                  group_size, weight_terms)

            module._modules[module_keys[-1]] = layer
            curr_layer += 1

    return model


def static_conv_layer_settings(model, weight_bits, group_size, num_terms):
    """(weight_bits, group_size, num_terms) per conv; the first conv, depthwise/grouped convs
    and squeeze-excite convs keep (16, 1, 16) (cnn_models/__init__.py:52-65)."""
    curr_layer = 0
    stats = []
    for name, layer in model.named_modules():
        if is_conv_layer(layer):
            if curr_layer == 0 or layer.groups > 1 or 'se' in name:
                stats.append((16, 1, 16))
                curr_layer += 1
                continue

            stats.append((weight_bits, group_size, num_terms))
            curr_layer += 1

    return stats


def convert_model(model, tr_params, data_bits, data_terms):
    # copy the model, since we modify it internally
    model = deepcopy(model)
    return replace_conv_layers(model, tr_params, data_bits, data_terms)
