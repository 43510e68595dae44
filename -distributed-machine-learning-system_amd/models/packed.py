"""Inference programs: reference modules -> BN-folded, MFMA-packed op lists.

``compile_model(module)`` turns an eval-mode ResNet / AlexNet into a flat list
of ops whose weights are laid out for the gfx950 implicit-GEMM kernel:

  * BatchNorm folded into the preceding conv: w' = w * g/sqrt(v+eps),
    b' = beta - mean * g/sqrt(v+eps)  ("BN folded into conv
    weights/bias at load time")
  * conv weights [Cout, Cin, KH, KW] -> [Cout, KH, KW, Cin] fp16 (K contiguous)
  * RGB stems (Cin = 3) -> [Cout, KH, ceil(KW/8)*8, 4] (one K-stage per kh row;
    fp32 programs: ceil(KW/4)*4 taps)
  * fp32 programs (dtype "fp32", the reference's precision) keep fp32 weights;
    their 3x3/stride-1 convs also carry the Winograd F(2x2,3x3) filter
    transform U = G g G^T [16, Cout, Cin] (conv_wino_f32.hip)
  * AlexNet fc6 columns permuted from NCHW-flatten to NHWC-flatten order
  * dropout elided (identity in eval), AdaptiveAvgPool(6,6) elided at 224 input

The same program runs on two executors: ``HipRunner`` (the real path, HIP
kernels, fp16 activations / fp32 accumulation, or all-fp32 for dtype
"fp32") and ``emulate`` (fp32 torch
re-execution of the *packed* weights — used on CPU to test folding/packing
without a GPU).
"""
from __future__ import annotations

import contextlib
import math
import os
import threading
from dataclasses import dataclass, field

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import reference as ref


@dataclass
class Conv:
    w: torch.Tensor          # packed [Cout, Kpad] fp16 (fp32 for dtype "fp32" programs)
    b: torch.Tensor          # [Cout] fp32
    cin: int
    cout: int
    kh: int
    kw: int
    stride: int
    pad: int
    relu: bool
    small: bool = False      # RGB stem packing
    wino: torch.Tensor | None = None   # fp32 3x3/s1: Winograd U = G g G^T [16, Cout, Cin]
    p3: torch.Tensor | None = None     # RGB stem on packed rows (pack_conv_weight_p3)
    sw: torch.Tensor | None = None     # fp32 programs: split-fp16 weights (pack_split_weight)
    s_scale: float = 1.0               # accumulator scale of ``sw`` / ``sp3`` (2^-e)
    sp3: torch.Tensor | None = None    # fp32 RGB stems: split-fp16 packed-row weights (pack_split_weight_p3)
    fs: torch.Tensor | None = None     # fp32 ResNet 7x7/2 stem: fused split stem weights (pack_stem_split)
    fs_bias: torch.Tensor | None = None  # ... its bias (with the normalisation shift folded in)
    fs_psum: torch.Tensor | None = None  # ... its border-correction prefix sums [8, 8, 64]
    fs_scale: float = 1.0              # ... its accumulator scale 2^-e

    def to(self, device):
        return Conv(self.w.to(device), self.b.to(device), self.cin, self.cout, self.kh, self.kw,
                    self.stride, self.pad, self.relu, self.small,
                    None if self.wino is None else self.wino.to(device),
                    None if self.p3 is None else self.p3.to(device),
                    None if self.sw is None else self.sw.to(device), self.s_scale,
                    None if self.sp3 is None else self.sp3.to(device),
                    None if self.fs is None else self.fs.to(device),
                    None if self.fs_bias is None else self.fs_bias.to(device),
                    None if self.fs_psum is None else self.fs_psum.to(device), self.fs_scale)

    @property
    def flops_per_out_pixel(self) -> int:
        return 2 * self.cin * self.kh * self.kw * self.cout


@dataclass
class Block:
    """Residual block: convs in order; the last conv fuses +identity and ReLU."""
    convs: list
    down: Conv | None = None

    def to(self, device):
        return Block([c.to(device) for c in self.convs], self.down.to(device) if self.down else None)


@dataclass
class Program:
    name: str
    kind: str                 # "resnet" | "alexnet"
    stem: Conv | None = None  # resnet
    blocks: list = field(default_factory=list)
    features: list = field(default_factory=list)  # alexnet: ("conv", Conv) | ("pool", (k, s, p))
    fcs: list = field(default_factory=list)       # list[Conv] as 1x1 convs (last -> fp32 logits)
    num_classes: int = 1000
    dtype: str = "fp16"       # activation / weight precision: "fp16" | "fp32" (reference precision)

    def to(self, device):
        p = Program(self.name, self.kind, self.stem.to(device) if self.stem else None,
                    [b.to(device) for b in self.blocks],
                    [(k, v.to(device) if k == "conv" else v) for k, v in self.features],
                    [f.to(device) for f in self.fcs], self.num_classes, self.dtype)
        return p

    def param_bytes(self) -> int:
        tot = 0
        for c in self.all_convs():
            tot += c.w.numel() * c.w.element_size() + c.b.numel() * 4
        return tot

    def all_convs(self):
        if self.stem is not None:
            yield self.stem
        for b in self.blocks:
            yield from b.convs
            if b.down is not None:
                yield b.down
        for k, v in self.features:
            if k == "conv":
                yield v
        yield from self.fcs


# ---------------------------------------------------------------------------
# packing
# ---------------------------------------------------------------------------

def fold_bn_f64(w: torch.Tensor, b: torch.Tensor | None, bn: nn.BatchNorm2d | None):
    """Fold an eval-mode BatchNorm into the preceding conv's (w, b), fp64 result."""
    w = w.detach().double()
    b = torch.zeros(w.shape[0], dtype=torch.float64) if b is None else b.detach().double()
    if bn is None:
        return w, b
    scale = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
    w = w * scale.view(-1, 1, 1, 1)
    b = (b - bn.running_mean.detach().double()) * scale + bn.bias.detach().double()
    return w, b


def fold_bn(w: torch.Tensor, b: torch.Tensor | None, bn: nn.BatchNorm2d | None):
    """Fold an eval-mode BatchNorm into the preceding conv's (w, b), in fp64."""
    w, b = fold_bn_f64(w, b, bn)
    return w.float(), b.float()


DTYPES = ("fp16", "fp32")


def pack_conv_weight(w: torch.Tensor, dtype: str = "fp16") -> tuple[torch.Tensor, bool]:
    """[Cout, Cin, KH, KW] fp32 -> packed [Cout, Kpad], small flag.

    fp16: small (Cin <= 4) rows are 8 taps x 4 channels (K stage of the f16
    kernels); big rows (kh, kw, c) with Cin % 64 == 0.
    fp32: small rows are 4 taps x 4 channels (one BK=16 stage of conv_f32.hip);
    big rows (kh, kw, c) with Cin % 16 == 0."""
    cout, cin, kh, kw = w.shape
    if dtype == "fp32":
        if cin <= 4:
            nsub = (kw + 3) // 4
            p = torch.zeros(cout, kh, nsub * 4, 4, dtype=torch.float32)
            p[:, :, :kw, :cin] = w.permute(0, 2, 3, 1)
            return p.reshape(cout, kh * nsub * 16).contiguous(), True
        if cin % 16 != 0:
            raise ValueError(f"Cin={cin} unsupported (need 3/4 or a multiple of 16)")
        return w.permute(0, 2, 3, 1).reshape(cout, kh * kw * cin).float().contiguous(), False
    if dtype != "fp16":
        raise ValueError(f"dtype must be one of {DTYPES}, got {dtype!r}")
    if cin <= 4:
        nsub = (kw + 7) // 8
        p = torch.zeros(cout, kh, nsub * 8, 4, dtype=torch.float32)
        p[:, :, :kw, :cin] = w.permute(0, 2, 3, 1)
        return p.reshape(cout, kh * nsub * 32).half().contiguous(), True
    if cin % 64 != 0:
        raise ValueError(f"Cin={cin} unsupported (need 3/4 or a multiple of 64)")
    return w.permute(0, 2, 3, 1).reshape(cout, kh * kw * cin).half().contiguous(), False


def pack_conv_weight_p3(w: torch.Tensor, dtype: str = "fp32") -> torch.Tensor:
    """[Cout, 3, KH, KW] -> packed-row stem weights: K = (kh, f) with
    f = 3*kw + c over cpk = ceil(3*KW/E) 16-byte chunks per kernel row
    (E = 4 fp32 / 8 fp16 elements; f >= 3*KW: zero), the order in which
    preprocess_pack3 lays a kernel row's pixels out; padded to whole K stages
    (16 fp32 = conv_f32.hip mode 2, 64 fp16 = conv_glds pack3)."""
    cout, cin, kh, kw = w.shape
    if cin != 3 or kw < 5:
        raise ValueError("packed-row stems take 3 input channels and KW >= 5")
    e, stage = (4, 16) if dtype == "fp32" else (8, 64)
    cpk = (3 * kw + e - 1) // e
    nk = (kh * cpk * e + stage - 1) // stage
    rows = torch.zeros(cout, kh, e * cpk, dtype=torch.float32)
    rows[:, :, :3 * kw] = w.float().permute(0, 2, 3, 1).reshape(cout, kh, 3 * kw)
    p = torch.zeros(cout, nk * stage, dtype=torch.float32)
    p[:, :kh * e * cpk] = rows.reshape(cout, -1)
    return p.contiguous() if dtype == "fp32" else p.half().contiguous()


def pack3_eligible(cin: int, kw: int, stride: int = 2, dtype: str = "fp32") -> bool:
    """fp32: any stride (<= 4 row copies); fp16 (8 halfs per chunk): stride
    even (2 or 4 row copies)."""
    return cin == 3 and kw >= 5 and (dtype == "fp32" or stride % 2 == 0)


def unpack_conv_weight(c: Conv) -> torch.Tensor:
    """Inverse of pack_conv_weight -> fp32 [Cout, Cin, KH, KW]."""
    w = c.w.float()
    if c.small:
        tpr = 4 if c.w.dtype == torch.float32 else 8        # taps per K row (see pack_conv_weight)
        nsub = (c.kw + tpr - 1) // tpr
        return w.view(c.cout, c.kh, nsub * tpr, 4)[:, :, :c.kw, :c.cin].permute(0, 3, 1, 2).contiguous()
    return w.view(c.cout, c.kh, c.kw, c.cin).permute(0, 3, 1, 2).contiguous()


# ---------------------------------------------------------------------------
# split fp16: fp32-accurate values as (hi, lo) half pairs (conv_glds SPLIT)
# ---------------------------------------------------------------------------
# A value v is carried as hi = fp16(v), lo = fp16(v - hi) (22 significant bits);
# a pixel of C channels is 2C halfs laid out [hi x32][lo x32] per 32 channels.
# The conv sums hi*hi + hi*lo + lo*hi on the f16 MFMA in f32.  Weights are
# pre-scaled by 2^e so that max |w| ~ 2^14 (their lo parts stay normal halfs);
# the kernel multiplies the accumulator by 2^-e.  On ResNet18 this is as
# accurate as fp32 (CPU emulation: 1.2e-7 relative logit error vs fp64, fp32
# itself 2.7e-7; tests/test_split.py).

SPLIT_BLOCK = 32


def split_eligible(cin: int, cout: int) -> bool:
    return cin % SPLIT_BLOCK == 0 and cout % SPLIT_BLOCK == 0


def to_split(x: torch.Tensor) -> torch.Tensor:
    """fp32 [..., C] -> split half [..., 2C] (C % 32 == 0)."""
    c = x.shape[-1]
    x = x.float()
    hi = x.half()
    lo = (x - hi.float()).half()
    blk = (*x.shape[:-1], c // SPLIT_BLOCK, 1, SPLIT_BLOCK)
    return torch.cat([hi.reshape(blk), lo.reshape(blk)], dim=-2).reshape(*x.shape[:-1], 2 * c)


def from_split(xs: torch.Tensor) -> torch.Tensor:
    """split half [..., 2C] -> fp32 [..., C] (hi + lo in f32)."""
    c = xs.shape[-1] // 2
    v = xs.float().reshape(*xs.shape[:-1], c // SPLIT_BLOCK, 2, SPLIT_BLOCK)
    return (v[..., 0, :] + v[..., 1, :]).reshape(*xs.shape[:-1], c)


def pack_split_weight(w: torch.Tensor) -> tuple[torch.Tensor, float]:
    """[Cout, Cin, KH, KW] -> (split weights [Cout, KH*KW*2*Cin] half, acc_scale).

    K order (kh, kw, 32-channel block, hi|lo, channel); the weights are scaled
    by 2^e (e from max |w|, so the largest is in [2^13, 2^14)) in fp64 before
    the split, acc_scale = 2^-e undoes it exactly in the epilogue."""
    cout, cin, kh, kw = w.shape
    if cin % SPLIT_BLOCK:
        raise ValueError(f"split weights need Cin % {SPLIT_BLOCK} == 0, got {cin}")
    e = _split_scale(w)
    ws = w.double().permute(0, 2, 3, 1) * (2.0 ** e)
    hi = ws.half()
    lo = (ws - hi.double()).half()
    blk = (cout, kh, kw, cin // SPLIT_BLOCK, 1, SPLIT_BLOCK)
    packed = torch.cat([hi.reshape(blk), lo.reshape(blk)], dim=4).reshape(cout, kh * kw * 2 * cin)
    return packed.contiguous(), 2.0 ** -e


def _split_scale(w: torch.Tensor) -> int:
    mx = float(w.abs().max())
    return 0 if mx == 0.0 else 14 - math.ceil(math.log2(mx))


def pack_split_weight_p3(w: torch.Tensor) -> tuple[torch.Tensor, float]:
    """RGB stem [Cout, 3, KH, KW] -> split-fp16 packed-row weights (conv_glds
    P3+SPLIT): K = (kh, f = 3*kw + c) over cpk = ceil(3*KW/8) 8-half chunks per
    kernel row (preprocess_pack3_split's order), padded to whole stages of 32
    K elements, each stage [hi x32][lo x32]; scaled by 2^e like pack_split_weight."""
    cout, cin, kh, kw = w.shape
    if cin != 3 or kw < 5:
        raise ValueError("packed-row stems take 3 input channels and KW >= 5")
    cpk = (3 * kw + 7) // 8
    k = kh * cpk * 8
    nk = (k + 31) // 32
    rows = torch.zeros(cout, kh, 8 * cpk, dtype=torch.float64)
    rows[:, :, :3 * kw] = w.double().permute(0, 2, 3, 1).reshape(cout, kh, 3 * kw)
    flat = torch.zeros(cout, nk * 32, dtype=torch.float64)
    flat[:, :k] = rows.reshape(cout, -1)
    e = _split_scale(w)
    flat = flat * (2.0 ** e)
    hi = flat.half()
    lo = (flat - hi.double()).half()
    packed = torch.cat([hi.reshape(cout, nk, 1, 32), lo.reshape(cout, nk, 1, 32)], dim=2).reshape(cout, nk * 64)
    return packed.contiguous(), 2.0 ** -e


def pack_stem_split(w: torch.Tensor, b: torch.Tensor | None = None):
    """ResNet stem [64, 3, 7, 7] (+ bias [64]) -> operands of the fused split stem
    (stem_fused.hip stem_split_kernel, exact-u8 form):

      fs     [2, 64, 7*32] half: hi and lo of w' = w * s_c, s_c = 1/(255 std_c),
             per kernel row 8 taps x 4 channels (tap 7, channel 3 zero), scaled
             by 2^e like pack_split_weight;
      scale  2^-e;
      bias   [64] f32: b + sum over all taps of w * c_c, c_c = -mean_c / std_c
             (the normalisation's shift for a pixel whose taps are all inside);
      psum   [8, 8, 64] f32: 2D prefix sums over (kh, kw) of sum_c w * c_c, from
             which the kernel corrects border pixels (zero padding in x, not u).

    conv(normalise(u)) = conv(w', u) + sum_{valid taps} w * c: u <= 255 is
    exact in fp16, so the B operand needs no lo part."""
    cout, cin, kh, kw = w.shape
    if (cout, cin, kh, kw) != (64, 3, 7, 7):
        raise ValueError("the fused split stem takes a [64, 3, 7, 7] conv")
    w = w.double()
    mean = torch.tensor(ref.IMAGENET_MEAN, dtype=torch.float64)
    std = torch.tensor(ref.IMAGENET_STD, dtype=torch.float64)
    ws = w * (1.0 / (255.0 * std)).view(1, 3, 1, 1)
    p = torch.zeros(cout, kh, 8, 4, dtype=torch.float64)
    p[:, :, :kw, :cin] = ws.permute(0, 2, 3, 1)
    e = _split_scale(ws)
    p = p.reshape(cout, kh * 32) * (2.0 ** e)
    hi = p.half()
    lo = (p - hi.double()).half()
    corr = (w * (-mean / std).view(1, 3, 1, 1)).sum(dim=1)            # [64, 7, 7]
    ps = torch.zeros(8, 8, cout, dtype=torch.float64)
    ps[1:, 1:] = corr.permute(1, 2, 0).cumsum(0).cumsum(1)
    bias = (torch.zeros(cout, dtype=torch.float64) if b is None else b.double()) + ps[7, 7]
    return torch.stack([hi, lo]).contiguous(), 2.0 ** -e, bias.float().contiguous(), ps.float().contiguous()


def alex_stem_k_index(kh: int, kw: int) -> tuple[int, int]:
    """(K step, slot of 8-k group base) of tap (kh, kw) in the fused AlexNet stem's
    K layout (alex_stem.hip): step kh holds taps 0..7 of row kh as 8 x 4 channels;
    tail step 11 + t holds taps 8, 9 (k 0..7) and 10 (k 8..11) of row 2t, and the
    same of row 2t + 1 at k 16..27.  Returns (step, k of channel 0)."""
    if kw < 8:
        return kh, 4 * kw
    t, second = divmod(kh, 2)
    base = 16 * second
    return 11 + t, base + (4 * (kw - 8) if kw < 10 else 8)


def pack_alex_stem_split(w: torch.Tensor, b: torch.Tensor | None = None):
    """AlexNet conv1 [64, 3, 11, 11] (+ bias) -> operands of the fused split
    AlexNet stem (alex_stem.hip alex_stem_split_kernel, exact-u8 form):

      fs     [2, 64, 17*32] half: hi and lo of w' = w * s_c, s_c = 1/(255 std_c),
             in the kernel's K layout (alex_stem_k_index), scaled by 2^e;
      scale  2^-e;
      bias   [64] f32: b + sum over all taps of w * c_c, c_c = -mean_c / std_c;
      psum   [12, 12, 64] f32: 2D prefix sums over (kh, kw) of sum_c w * c_c (border
             outputs get their in-image taps' sum from it)."""
    cout, cin, kh, kw = w.shape
    if (cout, cin, kh, kw) != (64, 3, 11, 11):
        raise ValueError("the fused split AlexNet stem takes a [64, 3, 11, 11] conv")
    w = w.double()
    mean = torch.tensor(ref.IMAGENET_MEAN, dtype=torch.float64)
    std = torch.tensor(ref.IMAGENET_STD, dtype=torch.float64)
    ws = w * (1.0 / (255.0 * std)).view(1, 3, 1, 1)
    p = torch.zeros(cout, 17, 32, dtype=torch.float64)
    for i in range(kh):
        for j in range(kw):
            st, k0 = alex_stem_k_index(i, j)
            p[:, st, k0:k0 + 3] = ws[:, :, i, j]
    e = _split_scale(ws)
    p = p.reshape(cout, 17 * 32) * (2.0 ** e)
    hi = p.half()
    lo = (p - hi.double()).half()
    corr = (w * (-mean / std).view(1, 3, 1, 1)).sum(dim=1)            # [64, 11, 11]
    ps = torch.zeros(12, 12, cout, dtype=torch.float64)
    ps[1:, 1:] = corr.permute(1, 2, 0).cumsum(0).cumsum(1)
    bias = (torch.zeros(cout, dtype=torch.float64) if b is None else b.double()) + ps[11, 11]
    return torch.stack([hi, lo]).contiguous(), 2.0 ** -e, bias.float().contiguous(), ps.float().contiguous()


def unpack_split_weight(c: "Conv") -> torch.Tensor:
    """Inverse of pack_split_weight -> fp32 [Cout, Cin, KH, KW] (hi + lo, unscaled)."""
    v = c.sw.double().reshape(c.cout, c.kh, c.kw, c.cin // SPLIT_BLOCK, 2, SPLIT_BLOCK)
    w = (v[..., 0, :] + v[..., 1, :]).reshape(c.cout, c.kh, c.kw, c.cin) * c.s_scale
    return w.permute(0, 3, 1, 2).float().contiguous()


# Winograd F(2x2, 3x3) filter transform (Lavin & Gray): U = G g G^T
WINO_G = torch.tensor([[1.0, 0.0, 0.0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0.0, 0.0, 1.0]], dtype=torch.float64)


def wino_weight(w: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, 3, 3] -> U [16, Cout, Cin] fp32, U[4i+j] = (G g G^T)[i][j],
    computed in fp64 and rounded once (conv_wino_f32.hip's A operand)."""
    assert w.shape[2:] == (3, 3)
    u = torch.einsum("ia,ocab,jb->ijoc", WINO_G, w.double(), WINO_G)
    return u.reshape(16, w.shape[0], w.shape[1]).float().contiguous()


def wino_eligible(cin: int, cout: int, kh: int, kw: int, stride: int, pad: int) -> bool:
    return kh == 3 and kw == 3 and stride == 1 and pad == 1 and cin % 16 == 0 and cout % 32 == 0


def make_conv(conv: nn.Conv2d, bn: nn.BatchNorm2d | None, relu: bool, dtype: str = "fp16") -> Conv:
    w, b = fold_bn(conv.weight, conv.bias, bn)
    pw, small = pack_conv_weight(w, dtype)
    sw, s_scale = None, 1.0
    if dtype == "fp32" and split_eligible(conv.in_channels, conv.out_channels):
        sw, s_scale = pack_split_weight(fold_bn_f64(conv.weight, conv.bias, bn)[0])
    if dtype == "fp32" and wino_eligible(conv.in_channels, conv.out_channels, *conv.kernel_size, conv.stride[0],
                                         conv.padding[0]):
        return Conv(pw, b.contiguous(), conv.in_channels, conv.out_channels, 3, 3, 1, 1, relu, small,
                    wino_weight(w), None, sw, s_scale)
    p3 = pack_conv_weight_p3(w, dtype) if pack3_eligible(conv.in_channels, conv.kernel_size[1], conv.stride[0], dtype) \
        else None
    sp3 = None
    if dtype == "fp32" and pack3_eligible(conv.in_channels, conv.kernel_size[1], conv.stride[0], "fp16") \
            and conv.out_channels % 64 == 0:
        sp3, s_scale = pack_split_weight_p3(fold_bn_f64(conv.weight, conv.bias, bn)[0])
    c = Conv(pw, b.contiguous(), conv.in_channels, conv.out_channels, conv.kernel_size[0],
             conv.kernel_size[1], conv.stride[0], conv.padding[0], relu, small, None, p3, sw, s_scale, sp3)
    if tuple(conv.weight.shape) == (64, 3, 7, 7) and conv.stride[0] == 2 and conv.padding[0] == 3:
        # the exact-u8 stem: split (fp32 programs) or its hi parts alone (fp16, ops.stem_u8_f16)
        c.fs, c.fs_scale, c.fs_bias, c.fs_psum = pack_stem_split(*fold_bn_f64(conv.weight, conv.bias, bn))
    elif tuple(conv.weight.shape) == (64, 3, 11, 11) and conv.stride[0] == 4 and conv.padding[0] == 2:
        # the fused AlexNet stem: split (ops.alex_stem_split) or its hi parts alone
        # (fp16 programs, ops.alex_stem_u8_f16)
        c.fs, c.fs_scale, c.fs_bias, c.fs_psum = pack_alex_stem_split(*fold_bn_f64(conv.weight, conv.bias, bn))
    return c


def make_fc(lin: nn.Linear, relu: bool, perm: torch.Tensor | None = None, dtype: str = "fp16") -> Conv:
    w = lin.weight.detach().float()
    if perm is not None:
        w = w[:, perm]
    k = w.shape[1]
    if k % 64 != 0:
        raise ValueError(f"FC in_features={k} must be a multiple of 64")
    sw, s_scale = None, 1.0
    if dtype == "fp32" and k % SPLIT_BLOCK == 0:
        w64 = lin.weight.detach().double()
        if perm is not None:
            w64 = w64[:, perm]
        sw, s_scale = pack_split_weight(w64.reshape(w.shape[0], k, 1, 1))
    return Conv((w if dtype == "fp32" else w.half()).contiguous(), lin.bias.detach().float().contiguous(), k, w.shape[0], 1, 1, 1,
                0, relu, False, sw=sw, s_scale=s_scale)


def compile_model(m: nn.Module, name: str, dtype: str = "fp16") -> Program:
    if dtype not in DTYPES:
        raise ValueError(f"dtype must be one of {DTYPES}, got {dtype!r}")
    m = m.eval()
    dt = dtype
    if isinstance(m, ref.ResNet):
        p = Program(name, "resnet", stem=make_conv(m.conv1, m.bn1, True, dt), dtype=dt)
        for li in range(1, 5):
            for blk in getattr(m, f"layer{li}"):
                down = make_conv(blk.downsample[0], blk.downsample[1], False, dt) if blk.downsample else None
                if isinstance(blk, ref.BasicBlock):
                    convs = [make_conv(blk.conv1, blk.bn1, True, dt), make_conv(blk.conv2, blk.bn2, True, dt)]
                else:
                    convs = [make_conv(blk.conv1, blk.bn1, True, dt), make_conv(blk.conv2, blk.bn2, True, dt),
                             make_conv(blk.conv3, blk.bn3, True, dt)]
                p.blocks.append(Block(convs, down))
        p.fcs = [make_fc(m.fc, False, dtype=dt)]
        p.num_classes = m.fc.out_features
        return p
    if isinstance(m, ref.AlexNet):
        p = Program(name, "alexnet", dtype=dt)
        mods = list(m.features)
        i = 0
        while i < len(mods):
            mod = mods[i]
            if isinstance(mod, nn.Conv2d):
                relu = i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
                p.features.append(("conv", make_conv(mod, None, relu, dt)))
                i += 2 if relu else 1
                continue
            if isinstance(mod, nn.MaxPool2d):
                p.features.append(("pool", (mod.kernel_size, mod.stride, mod.padding)))
            i += 1
        # NCHW flatten (c, h, w) -> our NHWC flatten (h, w, c)
        c, hw = 256, 36
        perm = torch.arange(c * hw).view(c, hw).t().reshape(-1)
        lins = [mm for mm in m.classifier if isinstance(mm, nn.Linear)]
        p.fcs = [make_fc(lins[0], True, perm, dt), make_fc(lins[1], True, dtype=dt),
                 make_fc(lins[2], False, dtype=dt)]
        p.num_classes = lins[2].out_features
        return p
    raise TypeError(f"cannot compile {type(m).__name__}")


def build_program(name: str, seed: int = 0, randomize_bn: bool = False, dtype: str = "fp16") -> Program:
    name = ref.canonical(name)
    return compile_model(ref.build(name, seed=seed, randomize_bn=randomize_bn), name, dtype)


# ---------------------------------------------------------------------------
# fp32 torch emulation of a packed program (CPU-testable)
# ---------------------------------------------------------------------------

def _emu_conv(c: Conv, x: torch.Tensor, res: torch.Tensor | None = None) -> torch.Tensor:
    y = F.conv2d(x, unpack_conv_weight(c).to(x.device), c.b.to(x.device), c.stride, c.pad)
    if res is not None:
        y = y + res
    return F.relu(y) if c.relu else y


@torch.no_grad()
def emulate(p: Program, img_u8: torch.Tensor) -> torch.Tensor:
    """fp32 logits of the packed program on NCHW torch ops."""
    x = ref.preprocess_u8(img_u8)
    if p.kind == "resnet":
        x = F.max_pool2d(_emu_conv(p.stem, x), 3, 2, 1)
        for blk in p.blocks:
            idt = x if blk.down is None else _emu_conv(blk.down, x)
            y = x
            for c in blk.convs[:-1]:
                y = _emu_conv(c, y)
            x = _emu_conv(blk.convs[-1], y, idt)
        x = x.mean(dim=(2, 3))
    else:
        for k, v in p.features:
            x = _emu_conv(v, x) if k == "conv" else F.max_pool2d(x, *v)
        x = x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)
    for fc in p.fcs:
        x = F.linear(x, fc.w.float().to(x.device), fc.b.to(x.device))
        if fc.relu:
            x = F.relu(x)
    return x


# ---------------------------------------------------------------------------
# HIP runner
# ---------------------------------------------------------------------------

_CAPTURE_LOCK = threading.Lock()


@contextlib.contextmanager
def _capture_nosync(g, device, pool=None):
    """``torch.cuda.graph(g, capture_error_mode="thread_local")`` without the
    device-wide synchronize (and gc / empty_cache) that context manager does
    first: a runtime that captures a graph for a new send slot while an RCCL
    collective of an earlier round is pending on a paused or dead member would
    wait for that collective -- until the backend's timeout (120 s) when the
    member was killed (bench --rehearse-rccl worker failover, round 5).  Work
    queued on the current stream is ordered before the capture by a stream
    dependency instead."""
    s = torch.cuda.Stream(device=device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        g.capture_begin(pool=pool, capture_error_mode="thread_local")
        try:
            yield
        finally:
            g.capture_end()
    torch.cuda.current_stream(device).wait_stream(s)


def x_is_cuda(t: torch.Tensor) -> bool:
    return t.is_cuda


class HipRunner:
    """Runs a packed Program through the gfx950 kernels.

    ``forward(img_u8)`` takes uint8 [B,224,224,3] on the GPU and returns
    (class int32 [B], prob fp32 [B]).  ``capture(batch)`` records the whole
    forward into a hipGraph (torch.cuda.CUDAGraph == hipGraph on ROCm) with a
    static input buffer, removing per-kernel launch overhead.
    """

    def __init__(self, program: Program, device=None, fuse_stem: bool = True, front_split: int | None = None,
                 winograd: bool = True, wino_variant: int | None = None, pack3: bool = True):
        from .. import ops

        ops.load()
        self.ops = ops
        self.fuse_stem = fuse_stem
        # fp32 3x3/s1 convs through the fused Winograd F(2x2,3x3) kernel (2.25x
        # fewer f32-MFMA products than the direct conv; conv_wino_f32.hip)
        self.winograd = winograd
        self.pack3 = pack3           # fp32 RGB stems on packed rows (conv_f32.hip mode 2)
        self.pack3_f16 = False       # fp16 AlexNet conv1 on packed rows (measured net-neutral, see _logits)
        self.side_down = False       # downsample conv on a second stream (A/B: tools/ab_flag.py --attr)
        self.stem_parts: int | None = None   # fp32 ResNet: stem + maxpool on batch parts (None = 1)
        # fp32 ResNets: residual stages on split-fp16 convs (conv_glds SPLIT:
        # hi*hi + hi*lo + lo*hi on the f16 MFMA, fp32-accurate) instead of the
        # f32-MFMA Winograd / direct kernels; False = the all-f32-MFMA path
        self.split = True
        # split path: fused stem + layer1 on this many batch parts (None = 1;
        # A/B: tools/ab_flag.py --attr split_front --values 1,2)
        self.split_front: int | None = None
        # split path: the batch as this many streams' halves (None = 1; A/B:
        # tools/ab_flag.py --attr split_streams --values 1,2)
        self.split_streams: int | None = None
        self._side: dict = {}
        # None = measured default (tools/wino_ablate.py, profiles/r2_v6_wino_variants.md):
        # variant 3 -- 4-wave blocks of 64 tiles, one 58-KiB LDS stage, two blocks
        # per CU -- is the fastest on every ResNet layer shape (same-box A/B:
        # 0.86-0.88x the 8-wave variant's time at 56/28/14, 0.67x at 7x7)
        self.wino_variant = wino_variant
        # >1: stem + the full-resolution blocks (ResNet layer1) run on this many
        # batch parts, each part's activations small enough to stay in the
        # 256 MiB Infinity Cache between the stem and the end of layer1.
        # None = measured default (tools/bench_split.py, profiles/r1_v8_front_split.log):
        # 2 parts for ResNet18/34 at >= 256 images (+1.3 %), else 1 (ResNet50: -0.6 %)
        self.front_split = front_split
        # >1: the WHOLE ResNet forward on this many batch parts, each part's
        # activations small enough to stay in the 256 MiB Infinity Cache from
        # producer to consumer (the memory-bound ResNet50 bottlenecks read every
        # 4x-wide tensor twice: next block's 1x1 reduce and its residual add).
        # None = measured default (_auto_batch_parts)
        self.batch_parts: int | None = None
        # split path: a stride-2 block's 1x1/2 downsample in the same launch as
        # its 3x3/2 conv (the downsample is that conv's centre tap; one input
        # read, one launch).  Measured slower (-2.1 / -3.1 % whole forward,
        # profiles/r3_dual_downsample.md), so off by default
        self.fuse_down = False
        self._dual: dict = {}
        # fp16 bottleneck blocks with a 1x1 downsample: the expansion 1x1 and the
        # downsample as ONE GEMM over [y | x] (ops.conv1x1_dual), so the
        # downsample's output (the residual) never reaches HBM
        self.fuse_down_1x1 = True
        self._dual1: dict = {}
        # fp16 ResNet50 layer1: a block's tail kernel also computes the next
        # block's reduce 1x1 from its output tile on chip (ops.conv1x1_fused_next)
        self.fuse_next_1x1 = True
        # fp16 ResNet stem in the exact-u8 form (stem_split_kernel<.., F16>: uint8 input exact, hi MFMA only);
        # off: the normalised-fp16 stem_fused_kernel is faster (ResNet18 -3.7 %, ResNet50 -1.8 %,
        # profiles/r3_ab_stem_u8_f16.md)
        self.stem_u8 = False
        # per-runner kernel routing for whole-graph A/Bs (ops.conv2d_split ``route``: bit 0 no
        # band-staged 3x3, bit 1 no row-streaming 64->64, bit 2 no streaming 1x1); 0 = defaults.
        # The kernel library itself has no process-global switches (VERDICT r4 weakness 4).
        self.route = 0
        self.device = torch.device(device or "cuda")
        self.p = program.to(self.device)
        self._graphs: dict[int, tuple] = {}
        # memory pool shared by this runner's captures (None: one private pool per
        # graph).  Sharing is safe only where every replay is stream-ordered on ONE
        # stream and a graph's outputs are consumed before another graph of the
        # pool replays (its intermediates may reuse their memory): HipExecutor
        # sets it (one private stream, outputs copied out or written to the
        # caller's buffer in the same stream order)
        self.graph_pool = None
        # split range guard: the split kernels set this flag
        # when an activation leaves fp16's range (|v| >= 65504 has no finite hi
        # half); softmax_top1 then marks the batch (class -2) and the eager
        # paths rerun it on the all-f32 kernels, which have fp32's range
        self._ovf = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.overflow_fallback = True
        self.overflow_reruns = 0
        self._capturing = False
        # replay captured graphs with a bare hipGraphLaunch (ops.graph_launch) instead of
        # torch.cuda.CUDAGraph.replay (tools/system_launch_probe.py measures both)
        self.direct_launch = os.environ.get("IDUNNO_DIRECT_LAUNCH", "0") == "1"

    # -- eager forward ------------------------------------------------------
    def _guarded(self) -> bool:
        return self.p.dtype == "fp32" and self.split and self._split_ok()

    def logits(self, img_u8: torch.Tensor, start: torch.Tensor | None = None, batch: int = -1,
               start_offset: int = 0) -> torch.Tensor:
        """fp32 logits.  With ``start`` (int64 GPU scalar) and ``batch``,
        ``img_u8`` is a whole HBM-resident shard and the images
        [*start - start_offset, ... + batch) are classified (device-side window).

        On the split path the range guard is armed; outside a graph capture a
        forward that tripped it is recomputed on the all-f32 kernels (one host
        read of the flag per eager call)."""
        if not self._guarded():
            return self._logits(img_u8, start, batch, start_offset)
        self._ovf.zero_()
        self.ops.set_split_guard(self._ovf)
        try:
            out = self._logits(img_u8, start, batch, start_offset)
        finally:
            self.ops.set_split_guard(None)
        if self.overflow_fallback and not self._capturing and int(self._ovf.item()):
            out = self.logits_f32_exact(img_u8, start, batch, start_offset)
            # these logits have fp32's range: a following softmax_top1 must not
            # mark the batch OVERFLOW_CLASS (forward() passes the flag on)
            self._ovf.zero_()
        return out

    def logits_f32_exact(self, img_u8, start=None, batch: int = -1, start_offset: int = 0):
        """The same forward on the all-f32-MFMA kernels (fp32 range)."""
        self.overflow_reruns += 1
        was = self.split
        self.split = False
        try:
            return self._logits(img_u8, start, batch, start_offset)
        finally:
            self.split = was

    def _auto_batch_parts(self, nb: int) -> int:
        return 1

    def _logits(self, img_u8: torch.Tensor, start: torch.Tensor | None = None, batch: int = -1,
                start_offset: int = 0) -> torch.Tensor:
        o = self.ops
        p = self.p
        native = tuple(img_u8.shape[1:3]) == (224, 224)
        if start is not None and not native:
            raise ValueError("device-side windows need 224x224 shards")
        nb = batch if start is not None else img_u8.shape[0]
        parts = self.batch_parts if self.batch_parts is not None else self._auto_batch_parts(nb)
        if p.kind == "resnet" and native and parts > 1 and nb >= 2 * parts:
            return self._logits_in_parts(img_u8, start, nb, start_offset, parts)
        if p.dtype == "fp32":
            return self._logits_f32(img_u8, start, batch, start_offset, native)
        s = p.stem
        fused = (self.fuse_stem and native and p.kind == "resnet" and s.small and s.kh == 7 and s.kw == 7
                 and s.stride == 2 and s.pad == 3 and s.cout == 64)
        first = p.features[0][1] if p.kind != "resnet" else None
        # AlexNet: uint8 -> conv1 + ReLU + max pool in one phased MFMA kernel (alex_stem.hip)
        astem = (first is not None and native and self.fuse_stem and first.fs is not None and first.kh == 11
                 and first.relu and len(p.features) > 1 and p.features[1][0] == "pool"
                 and tuple(p.features[1][1]) == (3, 2, 0))
        p3 = (first is not None and native and self.pack3_f16 and first.p3 is not None and not astem)
        if astem:
            x = o.alex_stem_u8_f16(img_u8, first.fs, first.fs_bias, first.fs_psum, first.fs_scale, start, batch,
                                   start_offset)
        elif p3:
            # AlexNet conv1 (11x11/4) on packed fp16 rows through conv_glds (K 448
            # vs 704 for NHWC4 on the register-staged conv_igemm): conv 290 -> 220
            # us at B=500, but the packed-row preprocess costs 133 vs 46 us, so it
            # is off by default (profiles/r2_v21_alexnet_f16_pack3.md)
            x3 = o.preprocess_pack3(img_u8, first.kw, first.stride, first.pad, start, batch, start_offset, f16=True)
            x = o.conv2d_pack3(x3, first.p3, first.b, img_u8.shape[2], first.kh, first.kw, first.stride, first.pad,
                               first.relu)
        elif not fused:
            x = o.preprocess(img_u8, start, batch, start_offset) if native else o.resize_crop(img_u8, 256, 224)
        feats = p.features[2:] if astem else (p.features[1:] if p3 else p.features)
        if p.kind == "resnet":
            nb = batch if start is not None else img_u8.shape[0]
            split = self.front_split if self.front_split is not None else \
                (2 if p.name in ("resnet18", "resnet34") and nb >= 256 else 1)
            nfront = self._front_blocks() if fused and split > 1 else 0
            if nfront:
                x = self._split_front(img_u8, start, batch, start_offset, nfront, split)
            elif fused:
                x = self._stem16(img_u8, start, batch, start_offset)
            else:
                x = o.conv2d(x, s.w, s.b, s.kh, s.kw, s.stride, s.pad, s.relu)
                x = o.maxpool2d(x, 3, 2, 1)
            x = self._blocks(p.blocks[nfront:], x)
            x = o.global_avgpool(x)
        else:
            for k, v in feats:
                if k == "conv":
                    x = o.conv2d(x, v.w, v.b, v.kh, v.kw, v.stride, v.pad, v.relu)
                else:
                    x = o.maxpool2d(x, *v)
            x = x.reshape(x.shape[0], -1)
        for i, fc in enumerate(p.fcs):
            last = i == len(p.fcs) - 1
            x = o.linear(x, fc.w, fc.b, relu=fc.relu, out_f32=last)
        return x

    def _logits_f32(self, img_u8, start, batch, start_offset, native):
        """Reference-precision forward: every activation, weight and product in
        fp32 (conv_f32.hip on the f32-input MFMA, elementwise_f32.hip)."""
        o, p = self.ops, self.p
        if not native:
            raise ValueError("the fp32 path takes 224x224 inputs (resize on host first)")
        first = p.stem if p.kind == "resnet" else p.features[0][1]
        nb = batch if start is not None else img_u8.shape[0]
        if p.kind == "resnet" and self.split and self._split_ok():
            # fused split stem (uint8 -> normalise -> conv7x7/2 -> ReLU -> max
            # pool, split out; or stem conv + max pool into the split layout)
            # -> split residual stages (the last conv writes fp32) -> fp32 avgpool / FC
            fused = self.fuse_stem and first.fs is not None and first.relu
            if fused and (self.split_streams or 1) > 1 and nb >= 64 and x_is_cuda(img_u8):
                return self._split_dual_stream(img_u8, start, batch, start_offset, nb)
            parts = self.split_front or 1
            nfront = self._front_blocks() if fused and parts > 1 and nb >= 2 * parts else 0
            if nfront:
                x = self._split_front_split(img_u8, start, batch, start_offset, nfront, parts)
            elif fused:
                x = o.stem_split(img_u8, first.fs, first.fs_bias, first.fs_psum, first.fs_scale, start, batch,
                                 start_offset)
            else:
                x = o.maxpool2d_split(self._stem_f32(first, img_u8, start, batch, start_offset), 3, 2, 1)
            for i, blk in enumerate(p.blocks[nfront:], nfront):
                x = self._block_split(blk, x, last=i == len(p.blocks) - 1)
            x = o.global_avgpool(x)
            for fc in p.fcs:
                x = o.linear(x, fc.w, fc.b, relu=fc.relu)
            return x
        parts = self.stem_parts if self.stem_parts is not None else 1
        if p.kind == "resnet" and parts > 1 and nb >= 2 * parts:
            # stem + maxpool on batch parts: a part's 112x112x64 stem output
            # (nb/parts x 3.2 MB) stays in the 256-MB Infinity Cache between the
            # conv's stores and the pool's reads instead of round-tripping HBM
            n = -(-nb // parts)
            x = None
            for sub in range(0, nb, n):
                m = min(n, nb - sub)
                if start is not None:
                    y = self._stem_f32(first, img_u8, start, m, start_offset, window=nb, sub=sub)
                else:
                    y = self._stem_f32(first, img_u8[sub:sub + m], None, -1, 0)
                if x is None:
                    x = torch.empty((nb, (y.shape[1] + 1) // 2, (y.shape[2] + 1) // 2, y.shape[3]),
                                    dtype=y.dtype, device=y.device)
                o.maxpool2d(y, 3, 2, 1, out=x[sub:sub + m])
            for blk in p.blocks:
                x = self._block(blk, x)
            x = o.global_avgpool(x)
            for fc in p.fcs:
                x = o.linear(x, fc.w, fc.b, relu=fc.relu)
            return x
        if p.kind == "alexnet" and self.split and self._split_ok():
            return self._alexnet_split(first, img_u8, start, batch, start_offset)
        x = self._stem_f32(first, img_u8, start, batch, start_offset)
        if p.kind == "resnet":
            x = o.maxpool2d(x, 3, 2, 1)
            for blk in p.blocks:
                x = self._block(blk, x)
            x = o.global_avgpool(x)
        else:
            for k, v in p.features[1:]:
                x = self._conv(v, x) if k == "conv" else o.maxpool2d(x, *v)
            x = x.reshape(x.shape[0], -1)
        for fc in p.fcs:
            x = o.linear(x, fc.w, fc.b, relu=fc.relu)
        return x

    def _logits_in_parts(self, img_u8, start, nb: int, start_offset: int, parts: int):
        """The whole forward on ``parts`` consecutive batch parts (same
        numbers as one pass: every op is per image)."""
        n = -(-nb // parts)
        outs = []
        keep = self.batch_parts
        self.batch_parts = 1
        try:
            for sub in range(0, nb, n):
                m = min(n, nb - sub)
                if start is None:
                    outs.append(self._logits(img_u8[sub:sub + m]))
                else:
                    outs.append(self._logits(img_u8, start + sub, m, start_offset))
        finally:
            self.batch_parts = keep
        return torch.cat(outs, 0)

    def _stem_f32(self, first, img_u8, start, batch, start_offset, window: int = -1, sub: int = 0):
        """fp32 RGB stem conv (+ReLU) of a window / part of the images."""
        o = self.ops
        if self.split and first.sp3 is not None:
            # split-fp16 packed rows (fp32-accurate) on the f16 MFMA, fp32 output
            x3 = o.preprocess_pack3_split(img_u8, first.kw, first.stride, first.pad, start, batch, start_offset,
                                          window, sub)
            return o.conv2d_pack3_split(x3, first.sp3, first.b, first.s_scale, img_u8.shape[2], first.kh, first.kw,
                                        first.stride, first.pad, first.relu)
        if self.pack3 and first.p3 is not None:
            # packed rows: K 176 vs 224 for the 7x7/2, 400 vs 528 for the 11x11/4
            x3 = o.preprocess_pack3(img_u8, first.kw, first.stride, first.pad, start, batch, start_offset, window,
                                    sub)
            return o.conv2d_pack3(x3, first.p3, first.b, img_u8.shape[2], first.kh, first.kw, first.stride,
                                  first.pad, first.relu)
        x = o.preprocess(img_u8, start, batch, start_offset, window, sub, f32=True)
        return o.conv2d(x, first.w, first.b, first.kh, first.kw, first.stride, first.pad, first.relu)

    def _conv(self, c, x, residual=None, out=None):
        if c.wino is not None and self.winograd and out is None and x.dtype == torch.float32 \
                and self.ops.wino_supported(x.shape[1], x.shape[2], c.cin, c.cout):
            var = self.wino_variant if self.wino_variant is not None else 3
            return self.ops.conv2d_wino(x, c.wino, c.b, c.relu, residual, var)
        return self.ops.conv2d(x, c.w, c.b, c.kh, c.kw, c.stride, c.pad, c.relu, residual=residual, out=out,
                               route=self.route | self._f16_route(x.shape[0]))

    def _f16_route(self, nb: int) -> int:
        """Measured per-model default on top of ``route``: ResNet50 fp16 at
        B >= 768 skips the band-staged 3x3 at W 28 (+1.2 % at B = 1024, -0.4 % at
        B = 400; ResNet18 fp16 keeps it: -0.7 % / -2.2 % without it at B = 400 /
        1024; profiles/r6q_ab_r50_route_0_1.log, profiles/r6r_*)."""
        return 1 if self.p.name == "resnet50" and nb >= 768 else 0

    def _blocks(self, blocks, x):
        """fp16 residual stages; with ``fuse_next_1x1`` a bottleneck block whose
        successor starts with a 1x1 reduce hands that conv's output over from
        its own tail kernel (ops.conv1x1_fused_next), and the successor skips it."""
        pre = None
        for i, blk in enumerate(blocks):
            nxt = blocks[i + 1] if i + 1 < len(blocks) else None
            x, pre = self._block_next(blk, x, pre, nxt)
        return x

    def _next_ok(self, blk, x, nxt) -> tuple | None:
        """(K2, stride) of a fusable tail + next reduce, else None."""
        if not (self.fuse_next_1x1 and nxt is not None and x.dtype == torch.float16 and x.is_cuda):
            return None
        last, d, r = blk.convs[-1], blk.down, nxt.convs[0]
        if not (last.kh == last.kw == 1 and last.stride == 1 and last.pad == 0 and r.kh == r.kw == 1
                and r.stride == 1 and r.pad == 0 and r.relu and last.relu and r.cin == last.cout):
            return None
        k2, stride = 0, 1
        if d is not None:
            if not (self.fuse_down_1x1 and d.kh == d.kw == 1 and d.pad == 0):
                return None
            k2, stride = d.cin, d.stride
        ho = (x.shape[1] - 1) // stride + 1
        ok = self.ops.load().conv1x1_fused_next_ok(last.cin, k2, last.cout, r.cout, x.shape[0] * ho * ho)
        return (k2, stride) if ok else None

    def _block_next(self, blk, x, pre, nxt):
        """(block output, the next block's first-conv output or None); ``pre`` =
        this block's first-conv output, already computed by the previous tail."""
        fused = self._next_ok(blk, x, nxt)
        if pre is None and fused is None:
            return self._block(blk, x), None
        y = pre if pre is not None else self._conv(blk.convs[0], x)
        for c in blk.convs[1:-1]:
            y = self._conv(c, y)
        if fused is None:
            last = blk.convs[-1]
            if self._dual1_ok(blk, x, None):
                w, b = self._dual1_weights(blk)
                return self.ops.conv1x1_dual(y, x, w, b, blk.down.stride, last.relu), None
            idt = x if blk.down is None else self._conv(blk.down, x)
            return self._conv(last, y, residual=idt), None
        r = nxt.convs[0]
        if blk.down is not None:
            w, b = self._dual1_weights(blk)
            out, z = self.ops.conv1x1_fused_next(y, w, b, r.w, r.b, x2=x, stride=fused[1])
        else:
            out, z = self.ops.conv1x1_fused_next(y, blk.convs[-1].w, blk.convs[-1].b, r.w, r.b, residual=x)
        return out, z

    def _dual1_ok(self, blk, x, out) -> bool:
        d, last = blk.down, blk.convs[-1]
        if not (self.fuse_down_1x1 and out is None and d is not None and x.dtype == torch.float16 and x.is_cuda):
            return False
        if not (last.kh == last.kw == 1 and last.stride == 1 and last.pad == 0 and d.kh == d.kw == 1 and d.pad == 0
                and not last.small and not d.small):
            return False
        ho = (x.shape[1] - 1) // d.stride + 1
        return bool(self.ops.load().conv1x1_dual_ok(last.cin, d.cin, last.cout, x.shape[0] * ho * ho))

    def _dual1_weights(self, blk):
        key = id(blk)
        if key not in self._dual1:
            last, d = blk.convs[-1], blk.down
            self._dual1[key] = (torch.cat([last.w, d.w], 1).contiguous(), (last.b + d.b).contiguous())
        return self._dual1[key]

    def _block(self, blk, x, out=None):
        """One residual block; the last conv fuses +identity and ReLU (into ``out``).
        With ``side_down`` the 1x1 downsample conv runs on a second stream,
        concurrently with the block's first conv (a fork/join that hipGraph
        capture keeps as two parallel branches)."""
        if self._dual1_ok(blk, x, out):
            y = x
            for c in blk.convs[:-1]:
                y = self._conv(c, y)
            w, b = self._dual1_weights(blk)
            return self.ops.conv1x1_dual(y, x, w, b, blk.down.stride, blk.convs[-1].relu)
        idt = x
        join = None
        if blk.down is not None:
            if self.side_down and x.is_cuda:
                cur = torch.cuda.current_stream(x.device)
                side = self._side_stream(x.device)
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    idt = self._conv(blk.down, x)
                x.record_stream(side)          # x / idt cross streams: keep the allocator honest
                idt.record_stream(cur)
                join = side
            else:
                idt = self._conv(blk.down, x)
        y = x
        for c in blk.convs[:-1]:
            y = self._conv(c, y)
        if join is not None:
            torch.cuda.current_stream(x.device).wait_stream(join)
        return self._conv(blk.convs[-1], y, residual=idt, out=out)

    def _capture_key(self, batch: int, packed=None, slot: int = 0):
        return ((batch if slot == 0 else (batch, slot)) if packed is None else ("pk", batch, packed.data_ptr()),
                self._variant())

    def has_graph(self, batch: int, packed=None, slot: int = 0) -> bool:
        """Whether ``capture(batch, packed=, slot=)`` would replay an existing graph."""
        return self._capture_key(batch, packed, slot) in self._graphs

    def _variant(self) -> tuple:
        """Kernel-choice switches a captured graph depends on (part of its cache key)."""
        return (self.split, self.split_front, self.split_streams, self.winograd, self.wino_variant, self.pack3,
                self.pack3_f16, self.side_down, self.stem_parts, self.front_split, self.fuse_stem, self.batch_parts,
                self.fuse_down, self.fuse_down_1x1, self.fuse_next_1x1, self.stem_u8, self.route)

    def _split_ok(self) -> bool:
        p = self.p
        if p.kind == "alexnet":
            return all(v.sw is not None for k, v in p.features[1:] if k == "conv") and \
                all(f.sw is not None for f in p.fcs)
        return all(c.sw is not None for b in p.blocks for c in [*b.convs, *([b.down] if b.down else [])])

    def _alexnet_split(self, first, img_u8, start, batch, start_offset):
        """fp32-accurate AlexNet: the fused split stem (uint8 -> conv1 + ReLU + max
        pool in one kernel, alex_stem.hip; without it: split packed-row conv1 with
        fp32 out, then the pool into the split layout) -> split convs 2-5 -> split
        FCs (split-K), fp32 logits."""
        o, p = self.ops, self.p
        feats = p.features[1:]
        if self.fuse_stem and first.fs is not None and first.kh == 11 and first.relu and feats \
                and feats[0][0] == "pool" and tuple(feats[0][1]) == (3, 2, 0):
            x = o.alex_stem_split(img_u8, first.fs, first.fs_bias, first.fs_psum, first.fs_scale, start, batch,
                                  start_offset)
            feats = feats[1:]
        else:
            x = self._stem_f32(first, img_u8, start, batch, start_offset)
        for k, v in feats:
            x = self._conv_split(v, x) if k == "conv" else o.maxpool2d_split(x, *v)
        x = x.reshape(x.shape[0], -1)         # split [B, 6*6*2*256]: the split layout of the NHWC flatten
        for i, fc in enumerate(p.fcs):
            x = o.linear_split(x, fc.sw, fc.b, fc.s_scale, relu=fc.relu, out_f32=i == len(p.fcs) - 1)
        return x

    def _conv_split(self, c, x, residual=None, out_f32=False, out=None):
        return self.ops.conv2d_split(x, c.sw, c.b, c.s_scale, c.kh, c.kw, c.stride, c.pad, c.relu, residual,
                                     out_f32, out=out, route=self.route)

    def _dual_ok(self, blk) -> bool:
        d, c0 = blk.down, blk.convs[0] if blk.convs else None
        return (self.fuse_down and d is not None and len(blk.convs) == 2 and c0.kh == 3 and c0.kw == 3
                and c0.pad == 1 and d.kh == 1 and d.kw == 1 and d.pad == 0 and d.stride == c0.stride
                and d.cin == c0.cin and d.cout == c0.cout and c0.relu and not d.relu
                and c0.sw is not None and d.sw is not None and c0.cout % 32 == 0)

    def _dual_weights(self, blk):
        """[2 Cout, 9*2C] split weights: the 3x3 conv's rows, then the 1x1
        downsample's rows in the centre-tap K block (zeros elsewhere)."""
        key = id(blk)
        got = self._dual.get(key)
        if got is None:
            c0, d = blk.convs[0], blk.down
            c2 = c0.sw.shape[1] // 9
            w = torch.zeros((2 * c0.cout, c0.sw.shape[1]), dtype=c0.sw.dtype, device=c0.sw.device)
            w[:c0.cout] = c0.sw
            w[c0.cout:, 4 * c2:5 * c2] = d.sw
            got = self._dual[key] = (w, torch.cat([c0.b, d.b]).contiguous())
        return got

    def _block_split(self, blk, x, last: bool = False, out=None):
        """Residual block on split-fp16 activations; with ``last`` the block's
        output is fp32 (for the avgpool / FC head); into ``out`` when given."""
        if self._dual_ok(blk):
            c0, d = blk.convs[0], blk.down
            w, b = self._dual_weights(blk)
            both = self.ops.conv2d_split_dual(x, w, b, c0.s_scale, d.s_scale, c0.cout, 3, 3, c0.stride, 1, True)
            y, idt = both[..., :2 * c0.cout], both[..., 2 * c0.cout:]
            return self._conv_split(blk.convs[1], y, residual=idt, out_f32=last, out=out)
        if not last and out is None and self._dual1_split_ok(blk, x):
            y = x
            for c in blk.convs[:-1]:
                y = self._conv_split(c, y)
            w, b, scale = self._dual1_split_weights(blk)
            return self.ops.conv1x1_dual_split(y, x, w, b, scale, blk.down.stride, blk.convs[-1].relu)
        idt = x if blk.down is None else self._conv_split(blk.down, x)
        y = x
        for c in blk.convs[:-1]:
            y = self._conv_split(c, y)
        return self._conv_split(blk.convs[-1], y, residual=idt, out_f32=last, out=out)

    def _dual1_split_ok(self, blk, x) -> bool:
        d, last = blk.down, blk.convs[-1]
        if not (self.fuse_down_1x1 and d is not None and x.is_cuda and last.sw is not None and d.sw is not None):
            return False
        if not (last.kh == last.kw == 1 and last.stride == 1 and last.pad == 0 and d.kh == d.kw == 1 and d.pad == 0):
            return False
        ho = (x.shape[1] - 1) // d.stride + 1
        return bool(self.ops.load().conv1x1_dual_split_ok(last.cin, d.cin, last.cout, x.shape[0] * ho * ho))

    def _dual1_split_weights(self, blk):
        """[W3 | Wds] re-packed as ONE split weight (one accumulator scale)."""
        key = ("split", id(blk))
        if key not in self._dual1:
            last, d = blk.convs[-1], blk.down
            w = torch.cat([unpack_split_weight(last).cpu(), unpack_split_weight(d).cpu()], 1)
            sw, scale = pack_split_weight(w)
            self._dual1[key] = (sw.to(self.device), (last.b + d.b).contiguous(), scale)
        return self._dual1[key]

    def _split_part(self, img_u8, start, nb, start_offset, window, sub):
        """Whole split ResNet forward of images [sub, sub + nb) of the window."""
        o, p, s = self.ops, self.p, self.p.stem
        if start is not None:
            x = o.stem_split(img_u8, s.fs, s.fs_bias, s.fs_psum, s.fs_scale, start, nb, start_offset,
                             window=window, sub=sub)
        else:
            x = o.stem_split(img_u8[sub:sub + nb], s.fs, s.fs_bias, s.fs_psum, s.fs_scale)
        for i, blk in enumerate(p.blocks):
            x = self._block_split(blk, x, last=i == len(p.blocks) - 1)
        x = o.global_avgpool(x)
        for fc in p.fcs:
            x = o.linear(x, fc.w, fc.b, relu=fc.relu)
        return x

    def _split_dual_stream(self, img_u8, start, batch, start_offset, nb):
        """The batch as two halves on two streams (fork/join, kept as parallel
        branches by hipGraph capture): one half's blocks fill the other's
        partial last wave of workgroups (layers 3-4 run 1.6-2.4 waves of blocks)."""
        cur = torch.cuda.current_stream(img_u8.device)
        side = self._side_stream(img_u8.device)
        side.wait_stream(cur)
        n0 = nb // 2
        window = nb if start is not None else -1
        l0 = self._split_part(img_u8, start, n0, start_offset, window, 0)
        with torch.cuda.stream(side):
            l1 = self._split_part(img_u8, start, nb - n0, start_offset, window, n0)
        img_u8.record_stream(side)
        l1.record_stream(cur)
        cur.wait_stream(side)
        return torch.cat([l0, l1])

    def _split_front_split(self, img_u8, start, batch, start_offset, nfront, parts):
        """Fused split stem + the first ``nfront`` (full-resolution) blocks on
        ``parts`` batch parts, so a part's activations can stay in the 256-MB
        Infinity Cache between kernels; the last block writes its slice of the
        full-batch output."""
        o, s = self.ops, self.p.stem
        B = batch if start is not None else img_u8.shape[0]
        n = -(-B // parts)
        out = None
        for sub in range(0, B, n):
            nb = min(n, B - sub)
            if start is not None:
                x = o.stem_split(img_u8, s.fs, s.fs_bias, s.fs_psum, s.fs_scale, start, nb, start_offset, window=B,
                                 sub=sub)
            else:
                x = o.stem_split(img_u8[sub:sub + nb], s.fs, s.fs_bias, s.fs_psum, s.fs_scale)
            for bi in range(nfront):
                blk = self.p.blocks[bi]
                if bi < nfront - 1:
                    x = self._block_split(blk, x)
                    continue
                if out is None:
                    out = torch.empty((B, x.shape[1], x.shape[2], 2 * blk.convs[-1].cout), dtype=torch.float16,
                                      device=x.device)
                self._block_split(blk, x, out=out[sub:sub + nb])
        return out

    def _side_stream(self, device):
        st = self._side.get(device)
        if st is None:
            st = self._side[device] = torch.cuda.Stream(device=device)
        return st

    def _front_blocks(self) -> int:
        """Leading blocks that keep the stem's resolution (ResNet layer1)."""
        n = 0
        for blk in self.p.blocks:
            if any(c.stride != 1 for c in blk.convs) or (blk.down is not None and blk.down.stride != 1):
                break
            n += 1
        return n

    def _stem16(self, img_u8, start, batch, start_offset, window: int = -1, sub: int = 0):
        """fp16 fused ResNet stem: the exact-u8 form (``stem_u8``) or the normalised-fp16 kernel."""
        o, s = self.ops, self.p.stem
        if self.stem_u8 and s.fs is not None:
            return o.stem_u8_f16(img_u8, s.fs, s.fs_bias, s.fs_psum, s.fs_scale, start, batch, start_offset,
                                 window=window, sub=sub)
        return o.stem_fused(img_u8, s.w, s.b, start, batch, start_offset, window=window, sub=sub)

    def _split_front(self, img_u8, start, batch, start_offset, nfront, split):
        """Stem + the first ``nfront`` blocks on ``split`` batch parts; the last
        block of each part writes its slice of the full-batch output."""
        o, s = self.ops, self.p.stem
        B = batch if start is not None else img_u8.shape[0]
        n = -(-B // split)
        out = None
        for sub in range(0, B, n):
            nb = min(n, B - sub)
            if start is not None:
                x = self._stem16(img_u8, start, nb, start_offset, window=B, sub=sub)
            else:
                x = self._stem16(img_u8[sub:sub + nb], None, -1, 0)
            for bi in range(nfront):
                blk = self.p.blocks[bi]
                if bi < nfront - 1:
                    x = self._block(blk, x)
                    continue
                if out is None:
                    c = blk.convs[-1]
                    out = torch.empty((B, x.shape[1], x.shape[2], c.cout), dtype=torch.float16, device=x.device)
                self._block(blk, x, out=out[sub:sub + nb])
        return out

    def forward(self, img_u8: torch.Tensor, start: torch.Tensor | None = None, batch: int = -1,
                start_offset: int = 0, packed: torch.Tensor | None = None):
        """(class int32 [B], prob fp32 [B]); with ``packed`` the fused
        softmax-top1 also writes (class, prob bits) pairs into it."""
        z = self.logits(img_u8, start, batch, start_offset)
        return self.ops.softmax_top1(z, packed, self._ovf if self._guarded() else None)

    __call__ = forward

    def has_window(self, shard: torch.Tensor, batch: int, packed: torch.Tensor | None = None) -> bool:
        """A window graph over ``shard`` (own start scalar) is already captured."""
        key = ("win", shard.data_ptr(), tuple(shard.shape), batch, None, 0,
               None if packed is None else packed.data_ptr(), self._variant())
        return key in self._graphs

    def capture_window(self, shard: torch.Tensor, batch: int, start: torch.Tensor | None = None,
                       start_offset: int = 0, packed: torch.Tensor | None = None):
        """hipGraph of forward over a device-side window of ``shard``.

        Returns (start, replay): write the first image index into the int64
        GPU scalar ``start`` (a stream-ordered device op, e.g. from an RCCL
        broadcast of the query descriptor), then ``replay()`` -> (cls, prob).
        No host round trip and no staging copy of the images.  A caller-owned
        ``start`` (e.g. the start field of this rank's row of the broadcast
        descriptor table) is read in place, minus ``start_offset``; with
        ``packed`` the graph also writes (class, prob bits) pairs there (the
        gather's send buffer)."""
        key = ("win", shard.data_ptr(), tuple(shard.shape), batch,
               None if start is None else start.data_ptr(), start_offset,
               None if packed is None else packed.data_ptr(), self._variant())
        if key in self._graphs:
            g, start, sout = self._graphs[key]
            return start, self._replayer(g, sout, shard)
        if start is None:
            start = torch.zeros(1, dtype=torch.int64, device=self.device)
        with _CAPTURE_LOCK:
            st = torch.cuda.Stream(device=self.device)
            st.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(st):
                self._capturing = True        # warm-up launches: no flag reads (a capture follows)
                try:
                    for _ in range(2):
                        self.forward(shard, start, batch, start_offset, packed)
                finally:
                    self._capturing = False
            torch.cuda.current_stream(self.device).wait_stream(st)
            g = torch.cuda.CUDAGraph()
            self._capturing = True
            try:
                with _capture_nosync(g, self.device, self.graph_pool):
                    sout = self.forward(shard, start, batch, start_offset, packed)
            finally:
                self._capturing = False
        self._graphs[key] = (g, start, sout)
        return start, self._replayer(g, sout, shard, packed)

    def _replayer(self, g, sout, *keep):
        """Replay closure that keeps this runner (its HBM-resident weights) and
        the captured inputs alive: the graph holds raw device pointers, so a
        caller that drops the runner and keeps only the closure must not let
        the weights go back to the allocator."""
        direct = self.direct_launch and hasattr(g, "raw_cuda_graph_exec")
        launch = self.ops.load().graph_launch if direct else None

        def replay():
            # several nodes may share a process (and a GPU): a replay while another
            # thread is capturing fails on ROCm ("prepare for replay during
            # capturing stage"), so replays and captures are mutually exclusive
            with _CAPTURE_LOCK:
                if direct:
                    launch(g.raw_cuda_graph_exec())      # hipGraphLaunch on the current stream only
                else:
                    g.replay()
            return sout
        replay._keep = (self, keep)
        return replay

    def close(self) -> None:
        """Destroy the captured graphs now, under the capture lock (a graph
        destroyed by another thread's garbage collection while a capture is
        active aborts the process: hipErrorStreamCaptureUnsupported)."""
        with _CAPTURE_LOCK:
            self._graphs.clear()
            import gc

            gc.collect()

    # -- hipGraph -------------------------------------------------------------
    def capture(self, batch: int, hw: int = 224, packed: torch.Tensor | None = None, slot: int = 0):
        """Capture forward for a fixed batch; returns (static_in, replay_fn).
        With ``packed`` the graph also writes (class, prob bits) pairs into
        that caller-owned buffer (e.g. a collective round's send buffer).
        ``slot`` > 0 captures an independent copy (own static buffers), so two
        forwards of the same batch size can be in flight."""
        key = self._capture_key(batch, packed, slot)
        if key in self._graphs:
            g, sin, sout = self._graphs[key]
            return sin, self._replayer(g, sout, packed)
        sin = torch.zeros(batch, hw, hw, 3, dtype=torch.uint8, device=self.device)
        with _CAPTURE_LOCK:  # one capture at a time per process; other threads keep launching
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                self._capturing = True
                try:
                    for _ in range(2):
                        self.forward(sin, packed=packed)
                finally:
                    self._capturing = False
            torch.cuda.current_stream(self.device).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            self._capturing = True
            try:
                with _capture_nosync(g, self.device, self.graph_pool):
                    sout = self.forward(sin, packed=packed)
            finally:
                self._capturing = False
        self._graphs[key] = (g, sin, sout)
        return sin, self._replayer(g, sout, packed)

    def flops_per_image(self) -> float:
        """Useful (unpadded) FLOPs for one 224x224 image."""
        return program_flops(self.p)


def program_flops(p: Program, hw: int = 224) -> float:
    """Analytic forward FLOPs per image (2*MAC, convs + FCs)."""
    tot = 0.0

    def out_hw(h, c):
        return (h + 2 * c.pad - c.kh) // c.stride + 1

    if p.kind == "resnet":
        h = out_hw(hw, p.stem)
        tot += h * h * p.stem.flops_per_out_pixel
        h = (h + 2 - 3) // 2 + 1
        for blk in p.blocks:
            hin = h
            for c in blk.convs:
                h = out_hw(h, c)
                tot += h * h * c.flops_per_out_pixel
            if blk.down is not None:
                hd = out_hw(hin, blk.down)
                tot += hd * hd * blk.down.flops_per_out_pixel
    else:
        h = hw
        for k, v in p.features:
            if k == "conv":
                h = out_hw(h, v)
                tot += h * h * v.flops_per_out_pixel
            else:
                kk, s, pp = v
                h = (h + 2 * pp - kk) // s + 1
    for fc in p.fcs:
        tot += fc.flops_per_out_pixel
    return tot
