"""EfficientNet-b0 with TensorFlow-style static "same" padding, module-for-module the
efficientnet_pytorch model the reference uses (cnn_models/__init__.py:16-25), including its
``Conv2dStaticSamePadding`` type (cnn_models/__init__.py:17,28; profile_model.py:3,57).

efficientnet_pytorch is not installed on this image, so the network is restated here with
the same module names (_conv_stem, _bn0, _blocks.N._expand_conv, ..._se_reduce, _conv_head,
_fc), so ``'se' in name`` and ``layer.groups > 1`` select the same (16, 1, 16) layers."""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


class Conv2dStaticSamePadding(nn.Conv2d):
    """Conv2d whose 'same' padding is fixed from the input image size at construction:
    pad = max((ceil(i/s) - 1)*s + (k-1)*d + 1 - i, 0), split left = pad//2, right = rest."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, image_size=None,
                 **kwargs):
        super(Conv2dStaticSamePadding, self).__init__(in_channels, out_channels, kernel_size,
                                                      stride, **kwargs)
        self.stride = self.stride if len(self.stride) == 2 else [self.stride[0]] * 2
        ih, iw = (image_size, image_size) if isinstance(image_size, int) else image_size
        kh, kw = self.weight.size()[-2:]
        sh, sw = self.stride
        oh, ow = math.ceil(ih / sh), math.ceil(iw / sw)
        pad_h = max((oh - 1) * self.stride[0] + (kh - 1) * self.dilation[0] + 1 - ih, 0)
        pad_w = max((ow - 1) * self.stride[1] + (kw - 1) * self.dilation[1] + 1 - iw, 0)
        if pad_h > 0 or pad_w > 0:
            self.static_padding = nn.ZeroPad2d((pad_w // 2, pad_w - pad_w // 2,
                                                pad_h // 2, pad_h - pad_h // 2))
        else:
            self.static_padding = nn.Identity()

    def forward(self, x):
        x = self.static_padding(x)
        return F.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation,
                        self.groups)


class MemoryEfficientSwish(nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(x)


def _out_size(image_size, stride):
    return int(math.ceil(image_size / stride))


class MBConvBlock(nn.Module):
    def __init__(self, inp, final_oup, kernel_size, stride, expand_ratio, se_ratio, image_size,
                 bn_mom=0.01, bn_eps=1e-3):
        super(MBConvBlock, self).__init__()
        self.id_skip = True
        self.stride = stride
        self.input_filters = inp
        self.output_filters = final_oup
        self.expand_ratio = expand_ratio
        self.has_se = se_ratio is not None and 0 < se_ratio <= 1
        oup = inp * expand_ratio
        if expand_ratio != 1:
            self._expand_conv = Conv2dStaticSamePadding(inp, oup, 1, bias=False,
                                                        image_size=image_size)
            self._bn0 = nn.BatchNorm2d(oup, momentum=bn_mom, eps=bn_eps)
        self._depthwise_conv = Conv2dStaticSamePadding(oup, oup, kernel_size, stride=stride,
                                                       groups=oup, bias=False,
                                                       image_size=image_size)
        self._bn1 = nn.BatchNorm2d(oup, momentum=bn_mom, eps=bn_eps)
        image_size = _out_size(image_size, stride)
        if self.has_se:
            num_squeezed = max(1, int(inp * se_ratio))
            self._se_reduce = Conv2dStaticSamePadding(oup, num_squeezed, 1, image_size=1)
            self._se_expand = Conv2dStaticSamePadding(num_squeezed, oup, 1, image_size=1)
        self._project_conv = Conv2dStaticSamePadding(oup, final_oup, 1, bias=False,
                                                     image_size=image_size)
        self._bn2 = nn.BatchNorm2d(final_oup, momentum=bn_mom, eps=bn_eps)
        self._swish = MemoryEfficientSwish()

    def forward(self, inputs):
        x = inputs
        if self.expand_ratio != 1:
            x = self._swish(self._bn0(self._expand_conv(inputs)))
        x = self._swish(self._bn1(self._depthwise_conv(x)))
        if self.has_se:
            x_sq = F.adaptive_avg_pool2d(x, 1)
            x_sq = self._se_expand(self._swish(self._se_reduce(x_sq)))
            x = torch.sigmoid(x_sq) * x
        x = self._bn2(self._project_conv(x))
        if self.id_skip and self.stride == 1 and self.input_filters == self.output_filters:
            x = x + inputs  # drop_connect is a no-op in eval mode
        return x


# (repeats, kernel, stride, expand, in, out, se) -- efficientnet-b0 block arguments
_B0_BLOCKS = [
    (1, 3, 1, 1, 32, 16, 0.25),
    (2, 3, 2, 6, 16, 24, 0.25),
    (2, 5, 2, 6, 24, 40, 0.25),
    (3, 3, 2, 6, 40, 80, 0.25),
    (3, 5, 1, 6, 80, 112, 0.25),
    (4, 5, 2, 6, 112, 192, 0.25),
    (1, 3, 1, 6, 192, 320, 0.25),
]


class EfficientNet(nn.Module):
    def __init__(self, num_classes=1000, image_size=224, dropout_rate=0.2):
        super(EfficientNet, self).__init__()
        bn_mom, bn_eps = 0.01, 1e-3
        self._conv_stem = Conv2dStaticSamePadding(3, 32, 3, stride=2, bias=False,
                                                  image_size=image_size)
        self._bn0 = nn.BatchNorm2d(32, momentum=bn_mom, eps=bn_eps)
        image_size = _out_size(image_size, 2)
        blocks = []
        for repeats, k, s, e, i, o, se in _B0_BLOCKS:
            blocks.append(MBConvBlock(i, o, k, s, e, se, image_size, bn_mom, bn_eps))
            image_size = _out_size(image_size, s)
            for _ in range(repeats - 1):
                blocks.append(MBConvBlock(o, o, k, 1, e, se, image_size, bn_mom, bn_eps))
        self._blocks = nn.ModuleList(blocks)
        self._conv_head = Conv2dStaticSamePadding(320, 1280, 1, bias=False,
                                                  image_size=image_size)
        self._bn1 = nn.BatchNorm2d(1280, momentum=bn_mom, eps=bn_eps)
        self._avg_pooling = nn.AdaptiveAvgPool2d(1)
        self._dropout = nn.Dropout(dropout_rate)
        self._fc = nn.Linear(1280, num_classes)
        self._swish = MemoryEfficientSwish()

    def forward(self, inputs):
        x = self._swish(self._bn0(self._conv_stem(inputs)))
        for block in self._blocks:
            x = block(x)
        x = self._swish(self._bn1(self._conv_head(x)))
        x = self._avg_pooling(x).flatten(start_dim=1)
        x = self._dropout(x)
        return self._fc(x)

    @staticmethod
    def get_image_size(model_name):
        return 224


def efficientnet_b0_model(num_classes=1000):
    return EfficientNet(num_classes=num_classes)
