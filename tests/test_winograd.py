"""Winograd F(2x2,3x3) math of conv_wino_f32.hip, re-done in torch on the CPU:
the packed filter transform (models.packed.wino_weight) + the kernel's input
(B^T d B) and output (A^T M A) transforms must reproduce F.conv2d (3x3, s1, p1),
in fp64 exactly (to rounding) and in fp32 to the fp32 tolerance the GPU test uses."""
import pytest
import torch
import torch.nn.functional as F

from idunno.models import packed


def wino_conv_reference(x, u, dtype):
    """x [B, C, H, W], u [16, Cout, C] -> [B, Cout, H, W] by 2x2 output tiles,
    with the same transforms and e = 4i + j order as the HIP kernel."""
    B, C, H, W = x.shape
    TY, TX = (H + 1) // 2, (W + 1) // 2
    xp = torch.zeros(B, C, 2 * TY + 2, 2 * TX + 2, dtype=dtype)
    xp[:, :, 1:H + 1, 1:W + 1] = x
    d = xp.unfold(2, 4, 2).unfold(3, 4, 2)             # [B, C, TY, TX, 4, 4]
    t = torch.stack([d[..., 0, :] - d[..., 2, :], d[..., 1, :] + d[..., 2, :],
                     d[..., 2, :] - d[..., 1, :], d[..., 1, :] - d[..., 3, :]], dim=-2)   # B^T d
    v = torch.stack([t[..., 0] - t[..., 2], t[..., 1] + t[..., 2],
                     t[..., 2] - t[..., 1], t[..., 1] - t[..., 3]], dim=-1)               # (B^T d) B
    v = v.reshape(B, C, TY, TX, 16)
    m = torch.einsum("eoc,bcyxe->boyxe", u.to(dtype), v).reshape(B, -1, TY, TX, 4, 4)
    t0 = m[..., 0, :] + m[..., 1, :] + m[..., 2, :]
    t1 = m[..., 1, :] - m[..., 2, :] - m[..., 3, :]
    y = torch.stack([torch.stack([t0[..., 0] + t0[..., 1] + t0[..., 2], t0[..., 1] - t0[..., 2] - t0[..., 3]], -1),
                     torch.stack([t1[..., 0] + t1[..., 1] + t1[..., 2], t1[..., 1] - t1[..., 2] - t1[..., 3]], -1)],
                    -2)                                   # [B, Cout, TY, TX, 2, 2]
    y = y.permute(0, 1, 2, 4, 3, 5).reshape(B, -1, 2 * TY, 2 * TX)
    return y[:, :, :H, :W]


@pytest.mark.parametrize("H,W,C,Cout", [(8, 8, 16, 32), (7, 7, 32, 64), (14, 5, 16, 32)])
def test_winograd_transforms_match_conv(H, W, C, Cout):
    torch.manual_seed(H * W + C)
    x = torch.randn(2, C, H, W, dtype=torch.float64)
    w = torch.randn(Cout, C, 3, 3, dtype=torch.float64)
    u = packed.wino_weight(w).double()
    ref = F.conv2d(x, w, None, 1, 1)
    y64 = wino_conv_reference(x, packed.wino_weight(w).double(), torch.float64)
    # U is rounded to fp32 once; everything else fp64
    assert (y64 - ref).abs().max().item() < 1e-5 * ref.abs().max().item()
    y32 = wino_conv_reference(x.float(), u.float(), torch.float32)
    assert (y32.double() - ref).abs().max().item() < 2e-5 * ref.abs().max().item()


def test_wino_weight_layout_and_eligibility():
    w = torch.randn(64, 48, 3, 3)
    u = packed.wino_weight(w)
    assert u.shape == (16, 64, 48) and u.dtype == torch.float32
    # e = 0 (i = j = 0) is g[0][0]; e = 15 (i = j = 3) is g[2][2]
    assert torch.allclose(u[0], w[:, :, 0, 0]) and torch.allclose(u[15], w[:, :, 2, 2])
    assert packed.wino_eligible(64, 64, 3, 3, 1, 1)
    assert not packed.wino_eligible(64, 64, 3, 3, 2, 1)
    assert not packed.wino_eligible(64, 20, 3, 3, 1, 1)
    p = packed.build_program("resnet18", dtype="fp32")
    n = sum(c.wino is not None for c in p.all_convs())
    assert n == 13          # every 3x3 stride-1 conv of ResNet18 (4 + 3 + 3 + 3)
    assert all(c.wino is None for c in packed.build_program("resnet18").all_convs())   # fp16: none
