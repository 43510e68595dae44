"""Band-staged split 3x3 conv (conv3x3_band.hip, tile 70): ResNet layers 2-4.

CPU: the patch LDS layout (chunk c of patch pixel t in slot c ^ (key(t) & 7),
key = row*(W+8) + col - 2W*segment) is conflict-free for every ds_read_b128 of
every tap, fragment and tile position the kernel issues.
GPU: the kernel against a float64 F.conv2d oracle of the same fp32 values (the
split path's 2e-5 tolerance), with partial last tiles, tiles that straddle
images, strided (in-place view) inputs / residuals, fp32 output, and a capped
persistent grid so one workgroup runs several tiles through one DMA ring.
"""
import pytest
import torch
import torch.nn.functional as F

from idunno.models import packed as P

DEV = "cuda"

# ds_read_b128 lane groups (MI355X_MICROARCH.md, LDS table): one LDS cycle each when conflict-free
GROUPS = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
GROUPS += [[lane + 32 for lane in g] for g in GROUPS]


def _tile_patch(W, BM, m0, M):
    """(b, oh, ow) of the tile's pixels and patch row of (b, ih), as the kernel builds them."""
    HW = W * W
    px = [divmod(min(m, M - 1), HW) for m in range(m0, m0 + BM)]
    px = [(b, r // W, r % W) for b, r in px]
    mlast = min(m0 + BM, M) - 1
    b0, oh0 = m0 // HW, (m0 % HW) // W
    b1, oh1 = mlast // HW, (mlast % HW) // W
    prow, r = {}, 0
    for seg, b in enumerate(range(b0, b1 + 1)):
        lo = oh0 if b == b0 else 0
        hi = oh1 if b == b1 else W - 1
        for ih in range(lo - 1, hi + 2):
            prow[(b, ih)] = (r, seg)
            r += 1
    return px, prow


@pytest.mark.parametrize("W,FM", [(28, 8), (14, 5), (7, 5), (56, 7)])
def test_band_patch_layout_conflict_free_cpu(W, FM):
    BM = 32 * FM
    M = 6 * W * W
    for m0 in range(0, M, BM):
        px, prow = _tile_patch(W, BM, m0, M)
        for f in range(BM // 16):
            for tap in range(9):
                kh, kw = divmod(tap, 3)
                for plane in (0, 4):
                    addr = []
                    for lane in range(64):
                        b, oh, ow = px[16 * f + (lane & 15)]
                        r, seg = prow[(b, oh + kh - 1)]
                        col = ow + kw
                        t, key = r * (W + 2) + col, r * (W + 8) + col - 2 * W * seg
                        c = (lane >> 4) + plane
                        addr.append(t * 128 + 16 * (c ^ (key & 7)))
                    for g in GROUPS:
                        slots = {}
                        for lane in g:
                            slots.setdefault((addr[lane] // 16) % 16, set()).add(addr[lane])
                        assert max(len(v) for v in slots.values()) == 1, (W, m0, f, tap, plane)


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------

@pytest.fixture(scope="module")
def ops():
    from idunno import ops as o

    o.load()
    return o


def _ref64(x, w, b, relu, res=None):
    y = F.conv2d(x.double().permute(0, 3, 1, 2), w.double().to(x.device), b.double().to(x.device), 1, 1)
    if res is not None:
        y = y + res.double().permute(0, 3, 1, 2)
    if relu:
        y = F.relu(y)
    return y.permute(0, 2, 3, 1)


def _check(y, ref, rel=2e-5):
    err = (y.double() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-12
    assert err <= rel * scale, f"max err {err:.3e} vs scale {scale:.3e} (rel {err / scale:.2e})"


BAND_CASES = [
    # (B, H, Cin, Cout): partial last tiles, tiles straddling images
    (2, 28, 128, 128),     # layer2: M 1568 = 6 tiles of 256 + 32
    (3, 14, 256, 256),     # layer3: 4 pixel tiles of 160 x 2 cout blocks
    (2, 28, 256, 128),
    (2, 14, 128, 256),
    (16, 28, 128, 128),    # 49 tiles
    (5, 7, 512, 512),      # layer4: M 245, 2 pixel tiles x 4 cout blocks
]


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,Cin,Cout", BAND_CASES)
@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("max_grid", [0, 3])
def test_band_conv_vs_fp64(ops, B, H, Cin, Cout, res, max_grid):
    torch.manual_seed(B * 31 + H + Cin + Cout + res)
    x = torch.randn(B, H, H, Cin, device=DEV)
    w = torch.randn(Cout, Cin, 3, 3) / (Cin * 9) ** 0.5
    b = torch.randn(Cout) * 0.1
    r = torch.randn(B, H, H, Cout, device=DEV) if res else None
    sw, scale = P.pack_split_weight(w)
    ext = ops.load()
    for relu in (True, False):
        y = ext.conv3x3_band_split(ops.split_from_f32(x), sw.to(DEV), b.to(DEV),
                                   None if r is None else ops.split_from_f32(r), relu, scale, False, max_grid)
        assert y.shape == (B, H, H, 2 * Cout)
        _check(P.from_split(y), _ref64(x, w, b, relu, r))


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,C", [(2, 28, 128), (3, 14, 256)])
def test_band_conv_out_f32_and_strided_views(ops, B, H, C):
    """fp32 output (the last block's conv), and x / residual read in place as the
    channel halves of one wider tensor (the dual conv's [y | downsample] output)."""
    torch.manual_seed(B + H + C)
    both = torch.randn(B, H, H, 2 * C, device=DEV)
    bs = ops.split_from_f32(both)                     # split [B, H, H, 4C]: [x | r] side by side
    xs, rs = bs[..., :2 * C], bs[..., 2 * C:]
    x, r = both[..., :C], both[..., C:]
    w = torch.randn(C, C, 3, 3) / (C * 9) ** 0.5
    b = torch.randn(C) * 0.1
    sw, scale = P.pack_split_weight(w)
    ext = ops.load()
    y = ext.conv3x3_band_split(xs, sw.to(DEV), b.to(DEV), rs, True, scale, True, 2)
    assert y.dtype == torch.float32 and y.shape == (B, H, H, C)
    _check(y, _ref64(x, w, b, True, r))
    y2 = ops.conv2d_split(xs, sw.to(DEV), b.to(DEV), scale, 3, 3, 1, 1, True, residual=rs, tile=70)
    _check(P.from_split(y2), _ref64(x, w, b, True, r))


@pytest.mark.gpu
def test_band_conv_matches_im2col_tile(ops):
    """Same conv through the band kernel and the 128x128 im2col split tile: both
    fp32-accurate, and agreeing to a few fp32 ulps of the output scale."""
    torch.manual_seed(3)
    B, H, C = 4, 28, 128
    x = ops.split_from_f32(torch.randn(B, H, H, C, device=DEV))
    w = torch.randn(C, C, 3, 3) / (C * 9) ** 0.5
    sw, scale = P.pack_split_weight(w)
    b = (torch.randn(C) * 0.1).to(DEV)
    y70 = P.from_split(ops.conv2d_split(x, sw.to(DEV), b, scale, 3, 3, 1, 1, True, tile=70)).double()
    y36 = P.from_split(ops.conv2d_split(x, sw.to(DEV), b, scale, 3, 3, 1, 1, True, tile=36)).double()
    assert (y70 - y36).abs().max().item() <= 2e-6 * y36.abs().max().item()


@pytest.mark.gpu
def test_band_conv_range_guard(ops):
    """A value past fp16's range sets the split guard flag (stored once per workgroup)."""
    torch.manual_seed(9)
    x = P.to_split(torch.rand(2, 14, 14, 128, device=DEV) * 0.1)
    sw, scale = P.pack_split_weight(torch.randn(128, 128, 3, 3) * 0.01)
    big = P.to_split(torch.full((2, 14, 14, 128), 65000.0, device=DEV))
    ext = ops.load()
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    ext.set_split_guard(flag)
    try:
        ext.conv3x3_band_split(x, sw.to(DEV), torch.zeros(128, device=DEV), None, True, scale, False, 0)
        torch.cuda.synchronize()
        assert flag.item() == 0
        ext.conv3x3_band_split(x, sw.to(DEV), torch.full((128,), 1000.0, device=DEV), big, True, scale, False, 0)
        torch.cuda.synchronize()
        assert flag.item() == 1
    finally:
        ext.set_split_guard(None)


# ---------------------------------------------------------------------------
# fp16 operands (ResNet50 b1024 / ResNet18 fp16 layers 2-4)
# ---------------------------------------------------------------------------

def _ref32_f16(x, w, b, relu, res=None):
    """fp32 oracle of the fp16 conv: the fp16 input / weight / residual values
    themselves, fp32 arithmetic."""
    y = F.conv2d(x.float().permute(0, 3, 1, 2), w.half().float().to(x.device), b.float().to(x.device), 1, 1)
    if res is not None:
        y = y + res.float().permute(0, 3, 1, 2)
    if relu:
        y = F.relu(y)
    return y.permute(0, 2, 3, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,Cin,Cout", BAND_CASES + [(3, 14, 512, 256)])
@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("max_grid", [0, 3])
def test_band_conv_f16_vs_fp32(ops, B, H, Cin, Cout, res, max_grid):
    torch.manual_seed(B * 17 + H + Cin + Cout + res)
    x = torch.randn(B, H, H, Cin, device=DEV).half()
    w = torch.randn(Cout, Cin, 3, 3) / (Cin * 9) ** 0.5
    b = torch.randn(Cout) * 0.1
    r = torch.randn(B, H, H, Cout, device=DEV).half() if res else None
    pw, small = P.pack_conv_weight(w, "fp16")
    assert not small
    ext = ops.load()
    for relu in (True, False):
        y = ext.conv3x3_band_f16(x, pw.to(DEV), b.to(DEV), r, relu, max_grid)
        assert y.dtype == torch.float16 and y.shape == (B, H, H, Cout)
        _check(y, _ref32_f16(x, w, b, relu, r).double(), rel=2e-3)


@pytest.mark.gpu
def test_band_conv_f16_matches_im2col_tile(ops):
    """fp16 conv2d through tile 70 (band) and the default im2col tile agree to fp16 rounding."""
    torch.manual_seed(5)
    B, H, C = 4, 28, 128
    x = torch.randn(B, H, H, C, device=DEV).half()
    w = torch.randn(C, C, 3, 3) / (C * 9) ** 0.5
    pw, _ = P.pack_conv_weight(w, "fp16")
    b = (torch.randn(C) * 0.1).to(DEV)
    r = torch.randn(B, H, H, C, device=DEV).half()
    y70 = ops.conv2d(x, pw.to(DEV), b, 3, 3, 1, 1, True, residual=r, tile=70).float()
    y42 = ops.conv2d(x, pw.to(DEV), b, 3, 3, 1, 1, True, residual=r, tile=36).float()
    assert (y70 - y42).abs().max().item() <= 2e-3 * y42.abs().max().item()
