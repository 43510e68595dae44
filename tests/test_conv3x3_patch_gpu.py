"""LDS-patch 3x3/s1 conv kernel (tile 40) vs a PyTorch fp32 reference, at the
ResNet 3x3 stride-1 shapes, partial row tiles (H=28 -> TH=8),
multi-image tiles (H=7 -> 4 images) with a partial last group, residual on/off."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = [pytest.mark.gpu, pytest.mark.experimental]
DEV = "cuda"


@pytest.mark.parametrize("B,H,C,Cout,res", [
    (2, 56, 64, 64, False), (2, 56, 64, 64, True), (2, 28, 128, 128, True), (3, 28, 64, 128, False),
    (2, 14, 256, 256, True), (5, 7, 512, 512, True), (3, 7, 512, 512, False), (1, 13, 192, 384, False),
])
def test_patch_conv_vs_fp32(B, H, C, Cout, res):
    from idunno import ops
    from idunno.models.packed import pack_conv_weight

    if not ops.load().has_experimental():
        pytest.skip("tile 40 lives in csrc/kernels/experimental/ (build with IDUNNO_EXPERIMENTAL=1)")
    torch.manual_seed(B * 7 + H + C + Cout)
    x = torch.randn(B, H, H, C, device=DEV).half()
    w = torch.randn(Cout, C, 3, 3) / (C * 9) ** 0.5
    b = torch.randn(Cout) * 0.1
    r = torch.randn(B, H, H, Cout, device=DEV).half() if res else None
    pw, _ = pack_conv_weight(w)
    y = ops.conv2d(x, pw.to(DEV), b.to(DEV), 3, 3, 1, 1, True, residual=r, tile=40)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.half().float().to(DEV), b.to(DEV), 1, 1)
    if r is not None:
        ref = ref + r.float().permute(0, 3, 1, 2)
    ref = F.relu(ref).permute(0, 2, 3, 1)
    scale = ref.abs().max().item()
    assert (y.float() - ref).abs().max().item() <= 1e-2 * scale + 1e-3
    # must agree with the im2col kernel bit-for-bit up to summation order
    y2 = ops.conv2d(x, pw.to(DEV), b.to(DEV), 3, 3, 1, 1, True, residual=r, tile=27)
    assert (y.float() - y2.float()).abs().max().item() <= 2e-3 * scale + 1e-3


@pytest.mark.parametrize("B,H,res", [(2, 56, False), (2, 56, True), (3, 30, True), (1, 9, False), (5, 57, True)])
def test_resident_weight_c64_conv_vs_fp32(B, H, res):
    """Tile 50 (conv3x3_c64.hip): all weights resident in LDS, persistent over
    8x28 output tiles with a double-buffered halo patch; partial tiles at the
    right / bottom edge (H = 30, 9, 57) and several tiles per workgroup (B = 5
    at H = 57 -> 80 tiles ... and B=2 at 56 -> 28 tiles)."""
    from idunno import ops
    from idunno.models.packed import pack_conv_weight

    torch.manual_seed(B * 11 + H)
    x = torch.randn(B, H, H, 64, device=DEV).half()
    w = torch.randn(64, 64, 3, 3) / (64 * 9) ** 0.5
    b = torch.randn(64) * 0.1
    r = torch.randn(B, H, H, 64, device=DEV).half() if res else None
    pw, _ = pack_conv_weight(w)
    y = ops.conv2d(x, pw.to(DEV), b.to(DEV), 3, 3, 1, 1, True, residual=r, tile=50)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.half().float().to(DEV), b.to(DEV), 1, 1)
    if r is not None:
        ref = ref + r.float().permute(0, 3, 1, 2)
    ref = F.relu(ref).permute(0, 2, 3, 1)
    scale = ref.abs().max().item()
    assert (y.float() - ref).abs().max().item() <= 1e-2 * scale + 1e-3
    y2 = ops.conv2d(x, pw.to(DEV), b.to(DEV), 3, 3, 1, 1, True, residual=r, tile=27)
    assert (y.float() - y2.float()).abs().max().item() <= 2e-3 * scale + 1e-3


def test_resident_weight_c64_many_tiles_per_workgroup():
    """B=400 layer1 shape: 5600 tiles over <= 256 persistent workgroups."""
    from idunno import ops
    from idunno.models.packed import pack_conv_weight

    torch.manual_seed(5)
    x = torch.randn(400, 56, 56, 64, device=DEV).half()
    w = torch.randn(64, 64, 3, 3) / (64 * 9) ** 0.5
    pw = pack_conv_weight(w)[0].to(DEV)
    b = (torch.randn(64) * 0.1).to(DEV)
    y = ops.conv2d(x, pw, b, 3, 3, 1, 1, True, tile=50)
    y2 = ops.conv2d(x, pw, b, 3, 3, 1, 1, True, tile=27)
    scale = y2.float().abs().max().item()
    assert (y.float() - y2.float()).abs().max().item() <= 2e-3 * scale + 1e-3
