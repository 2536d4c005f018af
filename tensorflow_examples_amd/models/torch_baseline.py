"""Stock PyTorch-ROCm eager ResNet-50/CIFAR (same architecture as models/resnet.py) used
ONLY as the labelled comparison point of bench.py ``--impl torch`` (the reference has no
published numbers: BASELINE.md §1).  Uses torch.nn + MIOpen convolutions, channels_last,
bf16 autocast, torch.optim.SGD(momentum, foreach) -- a typical "stock" training step.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class _Bottleneck(nn.Module):
    def __init__(self, cin, width, stride):
        super().__init__()
        cout = width * 4
        self.c1 = nn.Conv2d(cin, width, 1, bias=False)
        self.b1 = nn.BatchNorm2d(width)
        self.c2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.b2 = nn.BatchNorm2d(width)
        self.c3 = nn.Conv2d(width, cout, 1, bias=False)
        self.b3 = nn.BatchNorm2d(cout)
        self.proj = None
        if stride != 1 or cin != cout:
            self.proj = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        o = F.relu(self.b1(self.c1(x)))
        o = F.relu(self.b2(self.c2(o)))
        o = self.b3(self.c3(o))
        return F.relu(o + (x if self.proj is None else self.proj(x)))


class TorchResNet50Cifar(nn.Module):
    def __init__(self, num_classes=10):
        super().__init__()
        self.stem = nn.Conv2d(3, 64, 3, 1, 1, bias=False)
        self.bn = nn.BatchNorm2d(64)
        layers, cin = [], 64
        for si, n in enumerate([3, 4, 6, 3]):
            w = 64 * 2 ** si
            for bi in range(n):
                layers.append(_Bottleneck(cin, w, 2 if (bi == 0 and si > 0) else 1))
                cin = w * 4
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):
        x = F.relu(self.bn(self.stem(x)))
        x = self.layers(x)
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))
