"""Functional wrappers around the gfx950 HIP kernels (``idunno._C``).

Tensors are NHWC fp16 (or, for the reference-precision path, fp32) activations
on the current GPU.  Every function runs on
PyTorch's current HIP stream, so sequences of these ops can be captured into a
hipGraph with ``torch.cuda.graph``.
"""
from __future__ import annotations

from ._ext import available, load, so_path

__all__ = [
    "available", "load", "so_path", "conv2d", "linear", "preprocess", "resize_crop",
    "maxpool2d", "global_avgpool", "softmax_top1", "pick_tile", "pick_tile_f32", "synth_images", "stem_fused",
    "conv2d_wino", "wino_supported", "preprocess_pack3", "conv2d_pack3",
    "conv1x1_dual", "conv1x1_dual_split", "conv1x1_fused_next", "conv2d_split", "linear_split", "stem_split", "stem_u8_f16", "alex_stem_split", "alex_stem_u8_f16", "preprocess_pack3_split", "conv2d_pack3_split", "split_from_f32", "f32_from_split", "maxpool2d_split", "pick_tile_split",
]


def conv2d_split(x, w, bias, acc_scale: float, kh: int, kw: int, stride: int, pad: int, relu: bool,
                 residual=None, out_f32: bool = False, tile: int = -1, out=None, ksplit: int = -1, route: int = 0):
    """fp32-accurate conv on split-fp16 activations ([.., 2C] halfs, hi/lo per
    32 channels; models.packed.to_split) and weights (pack_split_weight):
    hi*hi + hi*lo + lo*hi on the f16 MFMA.  Output split (or fp32 with
    ``out_f32``).  ``tile`` forces a kernel (-1: the shape's default), ``ksplit``
    forces split-K slices (-1: auto for the default tile), ``route`` opts out of
    the specialised kernels (bit 0 band 3x3, bit 1 row-streaming 64->64, bit 2
    streaming 1x1; bit 3 restores the round-5 small-M rules for A/Bs) -- kernel
    choice depends on these arguments only."""
    return load().conv2d_split(x, w, bias, residual, kh, kw, stride, pad, relu, acc_scale, out_f32, tile, out,
                               ksplit, route)


def conv2d_split_dual(x, w, bias, acc_scale: float, acc_scale2: float, nsplit: int, kh: int, kw: int,
                      stride: int, pad: int, relu: bool, center_only: bool = True, tile: int = -1):
    """Two split convs of one input in one launch: output channels [0, nsplit)
    are conv 1 (``relu``, ``acc_scale``), the rest conv 2 (no ReLU,
    ``acc_scale2``; K over the centre tap only with ``center_only`` -- a 1x1
    stride-s conv is the centre tap of the 3x3 stride-s pad-1 conv).  Returns
    the [B, Ho, Wo, 2*Cout] split tensor; ``y[..., :2*nsplit]`` and
    ``y[..., 2*nsplit:]`` are the two convs' outputs (strided views that the
    split convs read in place)."""
    return load().conv2d_split_dual(x, w, bias, kh, kw, stride, pad, relu, acc_scale, acc_scale2, nsplit,
                                    center_only, tile)


def preprocess_pack3_split(img_u8, kw: int, stride: int, pad: int, start=None, batch: int = -1,
                           start_offset: int = 0, window: int = -1, sub: int = 0):
    """uint8 [B,H,W,3] -> split-fp16 packed-row stem input [B, H, 2*nc, wp]."""
    return load().preprocess_pack3_split(img_u8, kw, stride, pad, start, batch, start_offset, window, sub)


def conv2d_pack3_split(x3, w, bias, acc_scale: float, width: int, kh: int, kw: int, stride: int, pad: int,
                       relu: bool, tile: int = -1):
    """fp32-accurate RGB stem conv on split packed rows (conv_glds P3+SPLIT),
    fp32 output; ``w``, ``acc_scale`` = models.packed.pack_split_weight_p3(w)."""
    return load().conv2d_pack3_split(x3, w, bias, width, kh, kw, stride, pad, relu, acc_scale, tile)


def stem_split(img_u8, w, bias, psum, acc_scale: float, start=None, batch: int = -1, start_offset: int = 0,
               window: int = -1, sub: int = 0):
    """fp32-accurate fused ResNet stem on split fp16: uint8 [B,224,224,3] ->
    split [B,56,56,128] (normalise, conv 7x7/2 + bias, ReLU, max pool 3x3/2);
    ``w, acc_scale, bias, psum`` = models.packed.pack_stem_split(w, b)."""
    return load().stem_split(img_u8, w, bias, psum, acc_scale, start, batch, start_offset, window, sub)


def alex_stem_split(img_u8, w, bias, psum, acc_scale: float, start=None, batch: int = -1, start_offset: int = 0,
                    window: int = -1, sub: int = 0):
    """fp32-accurate fused AlexNet stem on split fp16: uint8 [B,224,224,3] ->
    split [B,27,27,128] (normalise, conv 11x11/4 pad 2 + bias, ReLU, max pool
    3x3/2); ``w, acc_scale, bias, psum`` = models.packed.pack_alex_stem_split(w, b)."""
    return load().alex_stem_split(img_u8, w, bias, psum, acc_scale, start, batch, start_offset, window, sub)


def alex_stem_u8_f16(img_u8, w, bias, psum, acc_scale: float, start=None, batch: int = -1, start_offset: int = 0,
                     window: int = -1, sub: int = 0):
    """fp16 fused AlexNet stem in the exact-u8 form (hi MFMA only): uint8
    [B,224,224,3] -> fp16 [B,27,27,64]; operands as ``alex_stem_split``."""
    return load().alex_stem_u8_f16(img_u8, w, bias, psum, acc_scale, start, batch, start_offset, window, sub)


def stem_u8_f16(img_u8, w, bias, psum, acc_scale: float, start=None, batch: int = -1, start_offset: int = 0,
                window: int = -1, sub: int = 0):
    """fp16 fused ResNet stem in the exact-u8 form: uint8 [B,224,224,3] -> fp16
    [B,56,56,64]; the weights of models.packed.pack_stem_split (hi parts used)."""
    return load().stem_u8_f16(img_u8, w, bias, psum, acc_scale, start, batch, start_offset, window, sub)


def split_linear_splits(m: int, k: int, n: int) -> int:
    """Split-K factor for a split-fp16 FC layer: ~1024 blocks of the default
    tile, slices of >= 512 input features, at most 8."""
    tiles = -(-m // 64) * (n // 128) if n % 128 == 0 else -(-m // 128) * -(-n // 64)
    s = 1
    while s < 8 and tiles * s < 1024 and k % (64 * s) == 0 and k // (2 * s) >= 512:
        s *= 2
    return s


def linear_split(x, w, bias, acc_scale: float, relu: bool = False, out_f32: bool = False, splits: int | None = None):
    """fp32-accurate y = act(x @ w.T + bias) on split fp16: x [M, 2K] split,
    w [N, 2K] split (models.packed.pack_split_weight of [N, K, 1, 1]); output
    split [M, 2N], or fp32 [M, N] with ``out_f32``.  K slices in one launch."""
    m, k2 = x.shape
    s = split_linear_splits(m, k2 // 2, w.shape[0]) if splits is None else splits
    return load().linear_split(x, w, bias, acc_scale, relu, out_f32, s, -1)


def split_from_f32(x):
    """fp32 [.., C] -> split-fp16 [.., 2C] on the GPU."""
    return load().split_from_f32(x)


def f32_from_split(x):
    """split-fp16 [.., 2C] -> fp32 [.., C] on the GPU."""
    return load().f32_from_split(x)


def maxpool2d_split(x, k: int, s: int, pad: int, out=None):
    """NHWC max pool of fp32 or split input into the split layout."""
    return load().maxpool2d_split(x, k, s, pad, out)


def pick_tile_split(m: int, cout: int) -> int:
    return int(load().pick_tile_split(m, cout))


def conv2d(x, w, bias, kh: int, kw: int, stride: int, pad: int, relu: bool,
           residual=None, out_f32: bool = False, tile: int = -1, out=None, ksplit: int = -1, route: int = 0):
    """Implicit-GEMM MFMA convolution with fused bias / residual / ReLU
    (into ``out`` when given: a contiguous NHWC tensor, e.g. a batch slice).

    fp16 activations -> f16 MFMA kernels (f32 accumulate); fp32 activations
    -> the reference-precision kernel on the f32-input MFMA (conv_f32.hip)."""
    import torch

    if x.dtype == torch.float32:
        return load().conv2d_nhwc_f32(x, w, bias, residual, kh, kw, stride, pad, relu, tile, out)
    return load().conv2d_nhwc(x, w, bias, residual, kh, kw, stride, pad, relu, out_f32, tile, out, ksplit, route)


def conv1x1_dual(x1, x2, w, bias, stride: int, relu: bool):
    """ResNet bottleneck tail as one GEMM (fp16): act([x1 | x2 at stride] . w^T
    + bias), w = [W_expand | W_downsample] (packed 1x1 weights side by side),
    bias = b_expand + b_downsample."""
    return load().conv1x1_dual(x1, x2, w, bias, stride, relu)


def conv1x1_fused_next(x1, w, bias, w2, b2, residual=None, x2=None, stride: int = 1, relu: bool = True):
    """Bottleneck tail and the next block's reduce 1x1 in one pass (fp16):
    y = act(x1 . w^T + bias + residual) -- or with ``x2`` (block input, at
    ``stride``) the dual form act([x1 | x2] . w^T + bias) -- and
    z = relu(y . w2^T + b2).  Returns (y, z)."""
    y, z = load().conv1x1_fused_next(x1, x2, w, bias, residual, w2, b2, stride, relu)
    return y, z


def conv1x1_dual_split(x1, x2, w, bias, acc_scale: float, stride: int, relu: bool):
    """Split-fp16 (fp32-accurate) form of ``conv1x1_dual``: split activations,
    w = pack_split_weight of [W_expand | W_downsample] (one ``acc_scale``)."""
    return load().conv1x1_dual_split(x1, x2, w, bias, acc_scale, stride, relu)


def conv2d_wino(x, u, bias, relu: bool, residual=None, variant: int = 0):
    """fp32 3x3/stride-1/pad-1 conv by fused Winograd F(2x2,3x3) (conv_wino_f32.hip);
    ``u`` = models.packed.wino_weight(w) [16, Cout, Cin]."""
    return load().conv2d_wino_f32(x, u, bias, residual, relu, variant)


def preprocess_pack3(img_u8, kw: int, stride: int, pad: int, start=None, batch: int = -1, start_offset: int = 0,
                     window: int = -1, sub: int = 0, f16: bool = False):
    """uint8 [B,H,W,3] -> packed-row stem input [B, H, nc, wp], fp32 (``f16``:
    fp16) (window args as ``preprocess``)."""
    return load().preprocess_pack3(img_u8, kw, stride, pad, start, batch, start_offset, window, sub, f16)


def conv2d_pack3(x3, w, bias, width: int, kh: int, kw: int, stride: int, pad: int, relu: bool, tile: int = -1):
    """RGB stem conv on packed rows (fp32: conv_f32 mode 2; fp16: conv_glds
    pack3); ``w`` = models.packed.pack_conv_weight_p3(w, dtype)."""
    return load().conv2d_pack3(x3, w, bias, width, kh, kw, stride, pad, relu, tile)


def wino_supported(h: int, w: int, cin: int, cout: int) -> bool:
    return cin % 16 == 0 and cout % 32 == 0 and bool(load().wino_supported(h, w, cin, cout))


# fp16 FC layers: K split into slices in ONE launch (conv_glds grid = tiles x
# slices, fp32 partials + combine) when the unsplit GEMM has few blocks.  The
# round-1 version issued one launch per slice and never paid
# (profiles/r1_v8_ab_linear_split.log); in one launch AlexNet fc6 101 -> 67 us,
# fc7 54 -> 37, fc8 40 -> 20 at B=500 (profiles/r2_v22_fc_f16_sweep.md).
# None = f16_linear_splits(); an int forces that split.
LINEAR_SPLITS: int | None = None


def f16_linear_splits(m: int, k: int, n: int) -> int:
    """Split factor for an fp16 FC layer: ~512 blocks of the default tile,
    at most 4 slices, slices of >= 1024 (short K does not pay the combine)."""
    tiles = (n // 128) * -(-m // 64) if n % 128 == 0 else -(-n // 64) * -(-m // 128)
    s = 1
    while s < 4 and tiles * s < 512 and k % (64 * 2 * s) == 0 and k // (2 * s) >= 1024:
        s *= 2
    return s


def f32_linear_splits(m: int, k: int, n: int) -> int:
    """Split-K factor for an fp32 FC layer: enough K slices (one launch, fp32
    partials + combine) for ~1024 blocks of 128x64 tiles, K slices >= 256.
    Measured (tools/fc_f32_sweep.py, profiles/r2_v16_fc_f32_sweep.md): AlexNet
    fc6 430 -> 339 us, fc8 178 -> 50 us; ResNet18 fc 26 -> 14 us; ResNet50 fc
    94 -> 54 us."""
    tiles = -(-n // 128) * -(-m // 64)
    s = 1
    while s < 8 and tiles * s < 1024 and k % (16 * 2 * s) == 0 and k // (2 * s) >= 256:
        s *= 2
    return s


def linear(x, w, bias, relu: bool = False, out_f32: bool = False, splits: int | None = None):
    """y = x @ w.T + bias: the conv kernel as a 1x1 conv on a 1x1 image, or
    with ``splits`` > 1 as split-K partial GEMMs + one combine kernel
    (fp32 ``x``: the f32 conv kernel, fp32 out)."""
    import torch

    b, k = x.shape
    n = w.shape[0]
    if x.dtype == torch.float32:
        s = f32_linear_splits(b, k, n) if splits is None else splits
        if s > 1:
            return load().linear_f32_splitk(x, w, bias, relu, s, -1)
        y = load().conv2d_nhwc_f32(x.view(b, 1, 1, k), w, bias, None, 1, 1, 1, 0, relu, -1, None)
        return y.view(b, n)
    if splits is None:
        splits = LINEAR_SPLITS if LINEAR_SPLITS is not None else f16_linear_splits(b, k, n)
    if splits > 1:
        return load().linear_splitk(x, w, bias, relu, out_f32, splits, -1)
    y = load().conv2d_nhwc(x.view(b, 1, 1, k), w, bias, None, 1, 1, 1, 0, relu, out_f32, -1, None)
    return y.view(b, n)


def preprocess(img_u8, start=None, batch: int = -1, start_offset: int = 0, window: int = -1, sub: int = 0,
               f32: bool = False):
    """uint8 [B,H,W,3] -> normalised fp16 (``f32``: fp32) [B,H,W,4] (4th channel zero).
    With ``start`` (int64 GPU scalar) and ``batch``, reads images
    [*start - start_offset, ... + batch) of the shard ``img_u8`` (device-side
    window; ``start`` may be a global image index and ``start_offset`` the
    shard's first global index).  A window of ``window`` images may be done
    in parts: this call covers images [sub, sub + batch) of it."""
    return load().preprocess(img_u8, start, batch, start_offset, window, sub, f32)


def resize_crop(img_u8, resize: int = 256, crop: int = 224):
    """Resize(shorter side) + CenterCrop + normalise, fused."""
    return load().resize_crop(img_u8, resize, crop)


def stem_fused(img_u8, w, bias, start=None, batch: int = -1, start_offset: int = 0, window: int = -1,
               sub: int = 0):
    """ResNet stem in one kernel: uint8 [B,H,W,3] -> fp16 [B,H/4,W/4,64]
    (optionally a device-side window of a shard, see ``preprocess``)."""
    return load().stem_fused(img_u8, w, bias, start, batch, start_offset, window, sub)


def maxpool2d(x, k: int = 3, s: int = 2, pad: int = 1, out=None):
    return load().maxpool2d_nhwc(x, k, s, pad, out)


def global_avgpool(x):
    return load().global_avgpool_nhwc(x)


def softmax_top1(logits, packed=None, ovf=None):
    """Returns (class int32 [B], probability fp32 [B]); with ``packed`` (int32
    [>= B, 2]) also writes (class, prob bits) pairs into it.  A set split
    range-guard flag ``ovf`` marks every row class -2 (OVERFLOW_CLASS)."""
    cls, prob = load().softmax_top1(logits, packed, ovf)
    return cls, prob


OVERFLOW_CLASS = -2      # softmax_top1's mark: a split activation left fp16's range


def set_split_guard(flag=None):
    """Split launches of this thread write their range-guard flag (int32
    device tensor) here; None turns the guard off."""
    load().set_split_guard(flag)


def pick_tile(m: int, cout: int) -> int:
    return int(load().pick_tile(m, cout))


def pick_tile_f32(m: int, cout: int, k: int, small: bool = False) -> int:
    """Default fp32 tile for an implicit GEMM of M pixels x Cout x K (= KH*KW*C)."""
    return int(load().pick_tile_f32(m, cout, k, small))


def synth_images(seed: int, start: int, n: int, device, hw: int = 224):
    """Deterministic synthetic uint8 images [n, hw, hw, 3] generated on the GPU
    (bit-identical to ``idunno.runtime.data.synth_images_cpu``)."""
    import torch

    return load().synth_images(int(seed), int(start), int(n), int(hw), torch.device(device))
