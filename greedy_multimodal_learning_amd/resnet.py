"""ResNet trunks with torchvision module/parameter names.

The reference calls `torchvision.models.resnet18(pretrained=False)` and uses
the trunk piecewise (src/model.py:53-56,65-106).  torchvision is not a
dependency here; this module provides the same architecture and the same
parameter names (`conv1`, `bn1`, `layer{1..4}.{i}.{conv,bn}{1,2}`,
`layer{2..4}.0.downsample.{0,1}`, `fc`), so checkpoints and the gating's
name-based grouping carry over unchanged.  Bottleneck/ResNet-50 serves
config C5.  Convolutions are `conv.GMConv2d` (bf16 MFMA kernels on HIP); batch
norms are `bn.GMBatchNorm2d`, which take the block's residual add and ReLU as
fused arguments (`relu` modules are kept for name/structure parity).
"""

import torch
import torch.nn as nn

from .bn import GMBatchNorm2d
from .conv import GMConv2d
from .gradsink import GradJoin

_JOIN = True


def _join():
    return GradJoin() if _JOIN else None
from .pool import GMMaxPool2d


def conv3x3(cin, cout, stride=1):
    return GMConv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def conv1x1(cin, cout, stride=1):
    return GMConv2d(cin, cout, 1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, cout, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(cin, cout, stride)
        self.bn1 = GMBatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(cout, cout)
        self.bn2 = GMBatchNorm2d(cout)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        # x feeds conv1 and the identity / downsample branch: their gradients are summed
        # inside the last consumer's backward kernel (gradsink.GradJoin), not by autograd
        join = _join()
        idt = x if self.downsample is None else self.downsample[1](self.downsample[0](x, grad_join=join))
        out = self.bn1(self.conv1(x, grad_join=join), relu=True)
        return self.bn2(self.conv2(out), residual=idt, relu=True,
                        residual_join=join if self.downsample is None else None)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv1x1(cin, planes)
        self.bn1 = GMBatchNorm2d(planes)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = GMBatchNorm2d(planes)
        self.conv3 = conv1x1(planes, planes * 4)
        self.bn3 = GMBatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        join = _join()
        idt = x if self.downsample is None else self.downsample[1](self.downsample[0](x, grad_join=join))
        out = self.bn1(self.conv1(x, grad_join=join), relu=True)
        out = self.bn2(self.conv2(out), relu=True)
        return self.bn3(self.conv3(out), residual=idt, relu=True,
                        residual_join=join if self.downsample is None else None)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = GMConv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = GMBatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = GMMaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                 GMBatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.bn1.relu_maxpool(self.conv1(x), self.maxpool)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet18(pretrained=False, **kw):
    if pretrained:
        raise RuntimeError("pretrained=True needs a torchvision weight download (unavailable offline)")
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet50(pretrained=False, **kw):
    if pretrained:
        raise RuntimeError("pretrained=True needs a torchvision weight download (unavailable offline)")
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)
