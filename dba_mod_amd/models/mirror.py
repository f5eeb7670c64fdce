"""Standard ``torch.nn`` definitions of the four reference architectures.

They serve three purposes and are *not* the compute path:

1. parameter initialisation identical to the reference (default PyTorch init; Kaiming-normal
   for the Tiny-ImageNet ResNet as in ``resnet_tinyimagenet.py:158-163``);
2. the ``state_dict`` key names/order, so checkpoints interchange with the reference
   (``helper.py:426-434``; ``shortcut.*`` vs ``downsample.*`` per model);
3. an autograd oracle for the functional program's forward/backward in the tests.

Architectures:
* ``MnistNet`` — ``MnistNet.py:7-31`` (conv5x5 1→20, conv5x5 20→50, fc 800→500→10,
  log_softmax);
* ``ResNet18Cifar`` — half-width ResNet-18, ``resnet_cifar.py:14-36,67-104``; the rest of the
  half-width CIFAR family (``ResNetCifar``: ResNet-34 with basic blocks, ResNet-50/101/152 with
  bottleneck blocks, ``resnet_cifar.py:39-64,106-116``) shares the key layout;
* ``ResNet18Tiny`` — torchvision-style ResNet-18 with a 200-way fc,
  ``resnet_tinyimagenet.py:40-77,122-238``;
* ``LoanNet`` — ``loan_model.py:10-27`` (91→46→23→9 MLP with dropout 0.5).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class MnistNet(nn.Module):
    def __init__(self) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(1, 20, 5, 1)
        self.conv2 = nn.Conv2d(20, 50, 5, 1)
        self.fc1 = nn.Linear(800, 500)
        self.fc2 = nn.Linear(500, 10)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = F.max_pool2d(F.relu(self.conv1(x)), 2, 2)
        x = F.max_pool2d(F.relu(self.conv2(x)), 2, 2)
        x = F.relu(self.fc1(x.flatten(1)))
        return F.log_softmax(self.fc2(x), dim=1)


class _CifarBlock(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.shortcut = nn.Sequential()
        if stride != 1 or cin != cout:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False),
                                          nn.BatchNorm2d(cout))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out)) + self.shortcut(x)
        return F.relu(out)


class _CifarBottleneck(nn.Module):
    """``resnet_cifar.py:39-64`` (expansion 4): 1x1 → 3x3(stride) → 1x1, projection shortcut."""
    expansion = 4

    def __init__(self, cin: int, planes: int, stride: int) -> None:
        super().__init__()
        cout = planes * self.expansion
        self.conv1 = nn.Conv2d(cin, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.shortcut = nn.Sequential()
        if stride != 1 or cin != cout:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False),
                                          nn.BatchNorm2d(cout))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out = F.relu(self.bn1(self.conv1(x)))
        out = F.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out)) + self.shortcut(x)
        return F.relu(out)


# CIFAR ResNet family of ``resnet_cifar.py:106-116``: arch -> (bottleneck?, blocks per stage)
CIFAR_RESNETS = {
    "resnet18_cifar": (False, (2, 2, 2, 2)),
    "resnet34_cifar": (False, (3, 4, 6, 3)),
    "resnet50_cifar": (True, (3, 4, 6, 3)),
    "resnet101_cifar": (True, (3, 4, 23, 3)),
    "resnet152_cifar": (True, (3, 8, 36, 3)),
}


class ResNetCifar(nn.Module):
    """Half-width CIFAR ResNet (stem 32, stages 32/64/128/256 x expansion), ``resnet_cifar.py:67-104``."""

    def __init__(self, bottleneck: bool = False, blocks=(2, 2, 2, 2), num_classes: int = 10) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(3, 32, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(32)
        exp = _CifarBottleneck.expansion if bottleneck else 1
        cin = 32
        for li, w in enumerate((32, 64, 128, 256)):
            layer = []
            for bi in range(blocks[li]):
                stride = 2 if (li > 0 and bi == 0) else 1
                layer.append(_CifarBottleneck(cin, w, stride) if bottleneck else _CifarBlock(cin, w, stride))
                cin = w * exp
            setattr(self, f"layer{li + 1}", nn.Sequential(*layer))
        self.linear = nn.Linear(256 * exp, num_classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out = F.relu(self.bn1(self.conv1(x)))
        for li in range(4):
            out = getattr(self, f"layer{li + 1}")(out)
        out = F.avg_pool2d(out, out.shape[-1])
        return self.linear(out.flatten(1))


class ResNet18Cifar(ResNetCifar):
    """Half-width ResNet-18 (stem 32, stages 32/64/128/256) — the reference's CIFAR model."""

    def __init__(self, num_classes: int = 10) -> None:
        super().__init__(False, (2, 2, 2, 2), num_classes)


class _TinyBlock(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False),
                                            nn.BatchNorm2d(cout))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + idt)


class ResNet18Tiny(nn.Module):
    """torchvision-layout ResNet-18, 7x7/2 stem + 3x3/2 maxpool, fc 512→200."""

    def __init__(self, num_classes: int = 200) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        cin = 64
        for li, w in enumerate((64, 128, 256, 512)):
            blocks = []
            for bi in range(2):
                stride = 2 if (li > 0 and bi == 0) else 1
                blocks.append(_TinyBlock(cin, w, stride))
                cin = w
            setattr(self, f"layer{li + 1}", nn.Sequential(*blocks))
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(512, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        for li in range(4):
            x = getattr(self, f"layer{li + 1}")(x)
        return self.fc(self.avgpool(x).flatten(1))


class LoanNet(nn.Module):
    def __init__(self, in_dim: int = 91, h1: int = 46, h2: int = 23, out_dim: int = 9) -> None:
        super().__init__()
        self.layer1 = nn.Sequential(nn.Linear(in_dim, h1), nn.Dropout(0.5), nn.ReLU())
        self.layer2 = nn.Sequential(nn.Linear(h1, h2), nn.Dropout(0.5), nn.ReLU())
        self.layer3 = nn.Sequential(nn.Linear(h2, out_dim))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.layer3(self.layer2(self.layer1(x)))


def build_mirror(arch: str) -> nn.Module:
    if arch in CIFAR_RESNETS:
        return ResNetCifar(*CIFAR_RESNETS[arch])
    return {"mnist": MnistNet, "resnet18_tiny": ResNet18Tiny, "loan": LoanNet}[arch]()
