"""DeepLabV3+ (ResNet-101 backbone, output stride 16) with the reference's parameter tree.

North star: the guided sampler's segmenter forward and input-gradient stay in PyTorch-ROCm; only the
gradient -> guidance update is a HIP kernel (``wc_sgg_update``).  This module is therefore plain
PyTorch, written so that its ``state_dict`` is key-for-key identical to the reference's
``seg_model.network.modeling.deeplabv3plus_resnet101`` (``modeling.py:193``, ``_segm_resnet`` :32-57,
``_deeplab.py:28-59,111-162``, ``utils.py:7-93``, ``backbone/resnet.py:121-213``) so that the
reference's trained checkpoints load.  No pretrained-backbone download path exists (offline build).
"""
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F


def _bn(c):
    return nn.BatchNorm2d(c)


class Bottleneck(nn.Module):
    """ResNet v1.5 bottleneck (stride on the 3x3), reference backbone/resnet.py:82-126."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, dilation=1):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = _bn(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=dilation, dilation=dilation, bias=False)
        self.bn2 = _bn(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = _bn(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        idt = x if self.downsample is None else self.downsample(x)
        return self.relu(out + idt)


class ResNetFeatures(nn.Module):
    """ResNet trunk up to layer4 (the IntermediateLayerGetter view, so no avgpool/fc keys)."""

    def __init__(self, layers=(3, 4, 23, 3), replace_stride_with_dilation=(False, False, True)):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = _bn(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self._inplanes, self._dilation = 64, 1
        self.layer1 = self._layer(64, layers[0], 1, False)
        self.layer2 = self._layer(128, layers[1], 2, replace_stride_with_dilation[0])
        self.layer3 = self._layer(256, layers[2], 2, replace_stride_with_dilation[1])
        self.layer4 = self._layer(512, layers[3], 2, replace_stride_with_dilation[2])

    def _layer(self, planes, blocks, stride, dilate):
        prev_dil = self._dilation
        if dilate:  # trade the stride for dilation (output stride control)
            self._dilation *= stride
            stride = 1
        down = None
        if stride != 1 or self._inplanes != planes * 4:
            down = nn.Sequential(nn.Conv2d(self._inplanes, planes * 4, 1, stride=stride, bias=False), _bn(planes * 4))
        mods = [Bottleneck(self._inplanes, planes, stride, down, prev_dil)]
        self._inplanes = planes * 4
        mods += [Bottleneck(self._inplanes, planes, dilation=self._dilation) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        low = self.layer1(x)
        x = self.layer4(self.layer3(self.layer2(low)))
        return OrderedDict(low_level=low, out=x)


def _conv_bn_relu(cin, cout, k=1, dilation=1):
    pad = 0 if k == 1 else dilation
    return [nn.Conv2d(cin, cout, k, padding=pad, dilation=dilation, bias=False), _bn(cout), nn.ReLU(inplace=True)]


class ASPPPooling(nn.Sequential):

    def __init__(self, cin, cout):
        super().__init__(nn.AdaptiveAvgPool2d(1), *_conv_bn_relu(cin, cout))

    def forward(self, x):
        size = x.shape[-2:]
        return F.interpolate(super().forward(x), size=size, mode='bilinear', align_corners=False)


class ASPP(nn.Module):

    def __init__(self, cin, rates):
        super().__init__()
        self.convs = nn.ModuleList([nn.Sequential(*_conv_bn_relu(cin, 256))] +
                                   [nn.Sequential(*_conv_bn_relu(cin, 256, 3, r)) for r in rates] +
                                   [ASPPPooling(cin, 256)])
        self.project = nn.Sequential(*_conv_bn_relu(5 * 256, 256), nn.Dropout(0.1))

    def forward(self, x):
        return self.project(torch.cat([c(x) for c in self.convs], dim=1))


class DeepLabHeadV3Plus(nn.Module):

    def __init__(self, in_channels, low_level_channels, num_classes, rates):
        super().__init__()
        self.project = nn.Sequential(*_conv_bn_relu(low_level_channels, 48))
        self.aspp = ASPP(in_channels, rates)
        self.classifier = nn.Sequential(*_conv_bn_relu(304, 256, 3), nn.Conv2d(256, num_classes, 1))

    def forward(self, feats):
        low = self.project(feats['low_level'])
        out = F.interpolate(self.aspp(feats['out']), size=low.shape[2:], mode='bilinear', align_corners=False)
        return self.classifier(torch.cat([low, out], dim=1))


class DeepLabV3(nn.Module):
    """backbone + head + bilinear resize to the input (reference utils.py:7-18)."""

    def __init__(self, backbone, classifier):
        super().__init__()
        self.backbone = backbone
        self.classifier = classifier

    def forward(self, x):
        return F.interpolate(self.classifier(self.backbone(x)), size=x.shape[-2:], mode='bilinear',
                             align_corners=False)


def deeplabv3plus_resnet101(num_classes: int = 19, output_stride: int = 16, pretrained_backbone: bool = False):
    """reference modeling.py:193 (``pretrained_backbone`` must be False: no network in this build)."""
    if pretrained_backbone:
        raise RuntimeError('pretrained backbone download is not available; load a checkpoint instead')
    dil, rates = ((False, True, True), (12, 24, 36)) if output_stride == 8 else ((False, False, True), (6, 12, 18))
    return DeepLabV3(ResNetFeatures((3, 4, 23, 3), dil), DeepLabHeadV3Plus(2048, 256, num_classes, rates))


def deeplabv3plus_resnet50(num_classes: int = 19, output_stride: int = 16, pretrained_backbone: bool = False):
    if pretrained_backbone:
        raise RuntimeError('pretrained backbone download is not available; load a checkpoint instead')
    dil, rates = ((False, True, True), (12, 24, 36)) if output_stride == 8 else ((False, False, True), (6, 12, 18))
    return DeepLabV3(ResNetFeatures((3, 4, 6, 3), dil), DeepLabHeadV3Plus(2048, 256, num_classes, rates))
