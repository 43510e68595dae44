"""fp16 resident-weight 3x3 64->64 conv (conv3x3_c64.hip, ResNet layer1).

CPU: the paired fragment map of the last x-tile (valid width 17..24, e.g.
columns 32..55 at W = 56) covers each of the tile's valid pixels exactly once,
and its ds_read_b128 B-fragment reads are conflict-free under the (row & 6)
chunk swizzle for every tap.
GPU: the kernel against an fp32 conv of the same fp16 values at widths that run
the paired mode (56, 52, 49, 24, 20) and the plain one (40, 33, 16), with and
without residual, and a batch that gives workgroups several tiles.
"""
import pytest
import torch
import torch.nn.functional as F

DEV = "cuda"
TH, TW, PW = 8, 32, 34
GROUPS = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
GROUPS += [[lane + 32 for lane in g] for g in GROUPS]


def _pix(fmx, wm, f, frow):
    """Tile-local (row, col) of lane frow of fragment f of wave wm (c64_pix)."""
    if fmx == 4:
        p = (wm * 4 + f) * 16 + frow
        return p // TW, p % TW
    k = wm * fmx + f
    if k < TH:
        return k, frow
    return 2 * (k - TH) + (frow >> 3), 16 + (frow if frow < 8 else (frow + 6) & 7)


def test_c64_paired_map_covers_tail_tile_cpu():
    seen = [_pix(3, wm, f, frow) for wm in range(4) for f in range(3) for frow in range(16)]
    assert len(set(seen)) == len(seen) == 8 * 24
    assert set(seen) == {(r, c) for r in range(8) for c in range(24)}


@pytest.mark.parametrize("fmx", [4, 3])
def test_c64_fragment_reads_conflict_free_cpu(fmx):
    for wm in range(4):
        for f in range(fmx):
            for tap in range(9):
                toff = (tap // 3) * PW + tap % 3
                for kk in (0, 1):
                    addr = []
                    for lane in range(64):
                        py, px = _pix(fmx, wm, f, lane & 15)
                        row = py * PW + px + toff
                        ch = (lane >> 4) + 4 * kk
                        addr.append(row * 128 + 16 * (ch ^ (row & 6)))
                    for g in GROUPS:
                        slots = [(addr[lane] // 16) % 16 for lane in g]
                        assert len(set(slots)) == 16, (fmx, wm, f, tap, kk)


@pytest.fixture(scope="module")
def ops():
    from idunno import ops as o

    o.load()
    return o


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,W", [(2, 56, 56), (3, 13, 52), (2, 9, 49), (1, 24, 24), (2, 11, 20),
                                   (2, 17, 40), (1, 8, 33), (2, 16, 16), (40, 56, 56)])
@pytest.mark.parametrize("res", [False, True])
def test_conv3x3_c64_f16_vs_fp32(ops, B, H, W, res):
    from idunno.models.packed import pack_conv_weight

    torch.manual_seed(B * 13 + H + W + res)
    x = torch.randn(B, H, W, 64, device=DEV).half()
    w = torch.randn(64, 64, 3, 3) / 24
    b = torch.randn(64) * 0.1
    r = torch.randn(B, H, W, 64, device=DEV).half() if res else None
    pw, _ = pack_conv_weight(w)
    for relu in (True, False):
        y = ops.conv2d(x, pw.to(DEV), b.to(DEV), 3, 3, 1, 1, relu, residual=r)
        ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.half().float().to(DEV), b.to(DEV), 1, 1)
        if r is not None:
            ref = ref + r.float().permute(0, 3, 1, 2)
        if relu:
            ref = F.relu(ref)
        ref = ref.permute(0, 2, 3, 1)
        err = (y.float() - ref).abs().max().item()
        assert err <= 2e-3 * ref.abs().max().item() + 1e-3, (err, B, H, W, res, relu)
