"""Plain-PyTorch definitions of the reference's model families (test oracle).

The reference loads ``torch.hub.load('pytorch/vision:v0.10.0', 'alexnet' |
'resnet18', pretrained=True)`` on every chunk (reference alexnet_resnet.py:17-22).
torchvision is not part of this framework; these modules re-state the same
architectures (torchvision v0.10 layer lists: SURVEY.md §2.4) with the same
``state_dict`` key names, so real pretrained weights saved as safetensors load
unchanged.  They are used

  * as the numerics oracle for the HIP kernels (fp32, CPU or GPU), and
  * as the CPU executor of the cluster when no GPU is present.

Random init follows torchvision's: kaiming-normal(fan_out) convs, BN
gamma=1/beta=0, running stats (0, 1); Linear default init.
"""
from __future__ import annotations

import threading

import torch
import torch.nn as nn
import torch.nn.functional as F


def _conv(cin, cout, k, s=1, p=0):
    return nn.Conv2d(cin, cout, k, stride=s, padding=p, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, width, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv(cin, width, 3, stride, 1)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = _conv(width, width, 3, 1, 1)
        self.bn2 = nn.BatchNorm2d(width)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return F.relu(y + idt)


class Bottleneck(nn.Module):
    """ResNet v1.5 bottleneck: the stride sits on the 3x3 conv."""

    expansion = 4

    def __init__(self, cin, width, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv(cin, width, 1)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = _conv(width, width, 3, stride, 1)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = _conv(width, width * 4, 1)
        self.bn3 = nn.BatchNorm2d(width * 4)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return F.relu(y + idt)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000):
        super().__init__()
        self.conv1 = _conv(3, 64, 7, 2, 3)
        self.bn1 = nn.BatchNorm2d(64)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        cin = 64
        for i, (n, width) in enumerate(zip(layers, (64, 128, 256, 512))):
            stride = 1 if i == 0 else 2
            blocks = []
            for j in range(n):
                s = stride if j == 0 else 1
                ds = None
                if j == 0 and (s != 1 or cin != width * block.expansion):
                    ds = nn.Sequential(_conv(cin, width * block.expansion, 1, s),
                                       nn.BatchNorm2d(width * block.expansion))
                blocks.append(block(cin, width, s, ds))
                cin = width * block.expansion
            setattr(self, f"layer{i + 1}", nn.Sequential(*blocks))
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(cin, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.maxpool(F.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


class AlexNet(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 64, 11, 4, 2), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2),
            nn.Conv2d(64, 192, 5, padding=2), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2),
            nn.Conv2d(192, 384, 3, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(384, 256, 3, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(256, 256, 3, padding=1), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2),
        )
        self.avgpool = nn.AdaptiveAvgPool2d((6, 6))
        self.classifier = nn.Sequential(
            nn.Dropout(), nn.Linear(256 * 36, 4096), nn.ReLU(inplace=True),
            nn.Dropout(), nn.Linear(4096, 4096), nn.ReLU(inplace=True),
            nn.Linear(4096, num_classes),
        )

    def forward(self, x):
        x = self.avgpool(self.features(x))
        return self.classifier(torch.flatten(x, 1))


def resnet18(num_classes=1000):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes)


def resnet34(num_classes=1000):
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes)


def resnet50(num_classes=1000):
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes)


def alexnet(num_classes=1000):
    return AlexNet(num_classes)


BUILDERS = {"resnet18": resnet18, "resnet34": resnet34, "resnet50": resnet50, "alexnet": alexnet}

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def preprocess_u8(img_u8: torch.Tensor) -> torch.Tensor:
    """uint8 [B,H,W,3] -> normalised fp32 NCHW (ToTensor + Normalize, reference
    alexnet_resnet.py:60-61)."""
    x = img_u8.permute(0, 3, 1, 2).float().div_(255.0)
    mean, std = _norm_consts(x.device)
    return (x - mean) / std


_NORM: dict = {}


def _norm_consts(device):
    """Per-device cached mean/std (no H2D copy inside a graph capture)."""
    key = str(device)
    if key not in _NORM:
        _NORM[key] = (torch.tensor(IMAGENET_MEAN, device=device).view(1, 3, 1, 1),
                      torch.tensor(IMAGENET_STD, device=device).view(1, 3, 1, 1))
    return _NORM[key]


_BUILD_LOCK = threading.Lock()


def build(name: str, seed: int = 0, randomize_bn: bool = False) -> nn.Module:
    """Random-init model of the named architecture, in eval mode.

    ``randomize_bn`` gives BN non-trivial affine params / running stats so the
    BN-folding path is actually exercised by the numerics tests.
    """
    name = canonical(name)
    g = torch.Generator().manual_seed(seed)
    # nn.init draws from the process-global CPU generator: nodes of one process
    # building models concurrently (LocalCluster threads) would interleave their
    # draws and get different weights for the same seed, so builds serialise.
    with _BUILD_LOCK, torch.random.fork_rng(devices=[]):
        torch.manual_seed(seed)
        m = BUILDERS[name]()
    if randomize_bn:
        for mod in m.modules():
            if isinstance(mod, nn.BatchNorm2d):
                c = mod.num_features
                mod.weight.data = 0.5 + torch.rand(c, generator=g)
                mod.bias.data = 0.2 * torch.randn(c, generator=g)
                mod.running_mean.data = 0.2 * torch.randn(c, generator=g)
                mod.running_var.data = 0.5 + torch.rand(c, generator=g)
    return m.eval()


ALIASES = {"resnet": "resnet18", "resnet-18": "resnet18", "resnet_18": "resnet18",
           "resnet-50": "resnet50", "alex": "alexnet"}


def canonical(name: str) -> str:
    """Canonical model name; accepts ``resnet`` as an alias for ``resnet18``
    (the reference's shell help says "alexnet or resnet", mp4_machinelearning.py:1126,
    while its batch/stat keys use "resnet18", :646, 1106 — SURVEY.md A15)."""
    n = name.strip().lower()
    n = ALIASES.get(n, n)
    if n not in BUILDERS:
        raise ValueError(f"unknown model {name!r}; known: {sorted(BUILDERS)}")
    return n
