"""Split-fp16 (fp32-accurate) path: layout helpers on the CPU, HIP kernels on the GPU.

A value v is carried as hi = fp16(v), lo = fp16(v - hi) (models/packed.py);
the conv (conv_glds SPLIT) sums hi*hi + hi*lo + lo*hi in f32 on the f16 MFMA.
The oracle is F.conv2d in float64 on the same fp32 inputs; the tolerance is
the fp32 path's (2e-5 of the output scale) -- the split path is held to fp32
accuracy, not fp16.
"""
import pytest
import torch
import torch.nn.functional as F

from idunno.models import packed as P

DEV = "cuda"


# ---------------------------------------------------------------------------
# CPU: layout, packing, emulated arithmetic
# ---------------------------------------------------------------------------

def test_split_roundtrip_cpu():
    torch.manual_seed(0)
    x = torch.randn(2, 5, 7, 96) * 3
    xs = P.to_split(x)
    assert xs.dtype == torch.float16 and xs.shape == (2, 5, 7, 192)
    # layout: block b of a pixel = [hi x32][lo x32]
    assert torch.equal(xs[..., :32], x[..., :32].half())
    assert torch.equal(xs[..., 64:96], x[..., 32:64].half())
    back = P.from_split(xs)
    # 22 significant bits; lo parts below fp16's normal range keep 2^-24 absolute
    assert bool(((back - x).abs() <= x.abs() * 2.0 ** -21 + 2.0 ** -24).all())


def test_pack_split_weight_cpu():
    torch.manual_seed(1)
    w = torch.randn(64, 96, 3, 3) * 0.03
    sw, scale = P.pack_split_weight(w)
    assert sw.shape == (64, 9 * 192) and sw.dtype == torch.float16
    # scale is a power of two, largest scaled weight in [2^13, 2^14)
    e = -torch.log2(torch.tensor(scale)).item()
    assert e == int(e)
    assert 2 ** 13 <= (w.abs().max() / scale).item() < 2 ** 14
    c = P.Conv(torch.empty(0), torch.zeros(64), 96, 64, 3, 3, 1, 1, False, sw=sw, s_scale=scale)
    back = P.unpack_split_weight(c)
    assert ((back - w).abs().max() / w.abs().max()).item() < 2.0 ** -22
    with pytest.raises(ValueError):
        P.pack_split_weight(torch.randn(8, 3, 7, 7))


def test_c64_split_lds_swizzle_conflict_free_cpu():
    """conv3x3_split.hip: chunk c of LDS column col in slot c ^ ((2*col) & 15);
    every ds_read_b128 lane group (lane = pixel + 16 * k-group) hits 16
    distinct 16-byte slots for every column base (tap shift) and chunk base."""
    groups = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
    groups += [[lane + 32 for lane in g] for g in groups]
    for base in range(16):
        for c0 in range(0, 16, 4):
            for g in groups:
                slots = {((c0 + (lane >> 4)) ^ ((2 * (base + (lane & 15))) & 15)) for lane in g}
                assert len(slots) == 16, (base, c0, g)


def test_c64_split_tail_fragment_conflict_free_cpu():
    """The tail fragment of a row pair: lanes 0-7 read columns 48.. of one ring
    row, lanes 8-15 the same columns of another (ring rows 60 * 256 B apart, a
    multiple of 16 slots): still 16 distinct 16-byte slots per lane group for
    every tap shift and chunk base."""
    groups = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
    groups += [[lane + 32 for lane in g] for g in groups]
    rb = 60 * 256
    for kw in range(3):
        for c0 in range(0, 16, 4):
            for ra, rbw in ((0, 1), (3, 4), (4, 0), (2, 2)):
                for g in groups:
                    addr = set()
                    for lane in g:
                        fr = lane & 15
                        col = 48 + (fr & 7) + kw
                        row = ra if fr < 8 else rbw
                        chunk = (c0 + (lane >> 4)) ^ ((2 * col) & 15)
                        addr.add(((row * rb + col * 256 + chunk * 16) // 16) % 16)
                    assert len(addr) == 16, (kw, c0, ra, rbw, g)


def _unpack_split_p3(sp3, scale, cout, kh, kw):
    cpk = (3 * kw + 7) // 8
    v = sp3.double().reshape(cout, -1, 2, 32)
    flat = (v[:, :, 0] + v[:, :, 1]).reshape(cout, -1)[:, :kh * cpk * 8] * scale
    return flat.reshape(cout, kh, 8 * cpk)[:, :, :3 * kw].reshape(cout, kh, kw, 3).permute(0, 3, 1, 2)


@pytest.mark.parametrize("kh,kw", [(7, 7), (11, 11)])
def test_pack_split_weight_p3_cpu(kh, kw):
    torch.manual_seed(kh)
    w = torch.randn(64, 3, kh, kw) * 0.05
    sp3, scale = P.pack_split_weight_p3(w)
    nk = (kh * ((3 * kw + 7) // 8) * 8 + 31) // 32
    assert sp3.shape == (64, nk * 64) and sp3.dtype == torch.float16
    back = _unpack_split_p3(sp3, scale, 64, kh, kw)
    assert ((back - w.double()).abs().max() / w.abs().max()).item() < 2.0 ** -22
    p = P.build_program("resnet18", dtype="fp32")
    assert p.stem.sp3 is not None
    assert P.build_program("alexnet", dtype="fp32").features[0][1].sp3 is not None
    assert p.stem.fs is not None and p.stem.fs.shape == (2, 64, 224)
    assert p.stem.fs_psum.shape == (8, 8, 64) and p.stem.fs_bias.shape == (64,)


def test_pack_stem_split_exact_u8_cpu():
    """conv(normalise(u)) == conv(w * s, u) + border-corrected sum of w * c (fp64)."""
    from idunno.models import reference as ref

    torch.manual_seed(3)
    w = torch.randn(64, 3, 7, 7) * 0.05
    b = torch.randn(64) * 0.1
    fs, scale, bias, psum = P.pack_stem_split(w, b)
    u = torch.randint(0, 256, (2, 30, 26, 3), dtype=torch.uint8)
    want = F.conv2d(ref.preprocess_u8(u).double(), w.double(), b.double(), 2, 3)
    v = fs.double().reshape(2, 64, 7, 8, 4)
    ws = ((v[0] + v[1]) * scale)[:, :, :7, :3].permute(0, 3, 1, 2)            # w * s_c [64, 3, 7, 7]
    got = F.conv2d(u.permute(0, 3, 1, 2).double(), ws, bias.double(), 2, 3)
    H, W = 30, 26
    for oy in range(got.shape[2]):
        hlo, hhi = max(0, 3 - 2 * oy), min(7, H + 3 - 2 * oy)
        for ox in range(got.shape[3]):
            wlo, whi = max(0, 3 - 2 * ox), min(7, W + 3 - 2 * ox)
            ps = psum.double()
            d = ps[hhi, whi] - ps[hlo, whi] - ps[hhi, wlo] + ps[hlo, wlo] - ps[7, 7]
            got[:, :, oy, ox] += d
    err = ((got - want).abs().max() / want.abs().max()).item()
    assert err < 1e-6, err


def test_pack_alex_stem_split_cpu():
    """The fused AlexNet stem's operands (K layout of alex_stem_k_index, exact-u8
    bias and border prefix sums) reproduce conv11x11/4(normalise(u)) in fp64."""
    from idunno.models import reference as ref

    torch.manual_seed(4)
    w = torch.randn(64, 3, 11, 11) * 0.03
    b = torch.randn(64) * 0.1
    fs, scale, bias, psum = P.pack_alex_stem_split(w, b)
    assert fs.shape == (2, 64, 17 * 32) and psum.shape == (12, 12, 64)
    v = ((fs[0].double() + fs[1].double()) * scale).reshape(64, 17, 32)
    ws = torch.zeros(64, 3, 11, 11, dtype=torch.float64)
    used = torch.zeros(17, 32, dtype=torch.bool)
    for i in range(11):
        for j in range(11):
            st, k0 = P.alex_stem_k_index(i, j)
            assert not used[st, k0:k0 + 4].any()
            used[st, k0:k0 + 4] = True
            ws[:, :, i, j] = v[:, st, k0:k0 + 3]
            assert (v[:, st, k0 + 3] == 0).all()              # the patch's 4th channel slot
    assert (v[:, ~used] == 0).all()                            # slots no tap owns hold zeros
    u = torch.randint(0, 256, (2, 47, 39, 3), dtype=torch.uint8)
    H, W = 47, 39
    want = F.conv2d(ref.preprocess_u8(u).double(), w.double(), b.double(), 4, 2)
    got = F.conv2d(u.permute(0, 3, 1, 2).double(), ws, bias.double(), 4, 2)
    ps = psum.double()
    for oy in range(got.shape[2]):
        hlo, hhi = max(0, 2 - 4 * oy), min(11, H + 2 - 4 * oy)
        for ox in range(got.shape[3]):
            wlo, whi = max(0, 2 - 4 * ox), min(11, W + 2 - 4 * ox)
            got[:, :, oy, ox] += ps[hhi, whi] - ps[hlo, whi] - ps[hhi, wlo] + ps[hlo, wlo] - ps[11, 11]
    err = ((got - want).abs().max() / want.abs().max()).item()
    assert err < 1e-6, err


def _emu_split_conv(x, sw, scale, cout, cin, k, stride, pad):
    """The kernel's arithmetic in fp64 on CPU: hi*hi + hi*lo + lo*hi."""
    xs = P.to_split(x).double().reshape(*x.shape[:-1], cin // 32, 2, 32)
    xh = xs[..., 0, :].reshape(x.shape).permute(0, 3, 1, 2)
    xl = xs[..., 1, :].reshape(x.shape).permute(0, 3, 1, 2)
    ws = sw.double().reshape(cout, k, k, cin // 32, 2, 32)
    wh = ws[..., 0, :].reshape(cout, k, k, cin).permute(0, 3, 1, 2)
    wl = ws[..., 1, :].reshape(cout, k, k, cin).permute(0, 3, 1, 2)
    y = F.conv2d(xh, wh, None, stride, pad) + F.conv2d(xh, wl, None, stride, pad) + F.conv2d(xl, wh, None, stride, pad)
    return y * scale


def test_split_arithmetic_matches_fp32_accuracy_cpu():
    torch.manual_seed(2)
    x = F.relu(torch.randn(2, 12, 12, 64))
    w = torch.randn(32, 64, 3, 3) / 24
    sw, scale = P.pack_split_weight(w)
    y = _emu_split_conv(x, sw, scale, 32, 64, 3, 1, 1)
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), None, 1, 1)
    y32 = F.conv2d(x.permute(0, 3, 1, 2), w, None, 1, 1).double()
    err = ((y - ref).abs().max() / ref.abs().max()).item()
    err32 = ((y32 - ref).abs().max() / ref.abs().max()).item()
    assert err < 4 * max(err32, 1e-7), (err, err32)


def test_compile_fp32_program_has_split_weights_cpu():
    p = P.build_program("resnet18", dtype="fp32")
    convs = [c for b in p.blocks for c in [*b.convs, *([b.down] if b.down else [])]]
    assert convs and all(c.sw is not None for c in convs)
    assert p.stem.sw is None        # C = 3 stem stays on the f32 MFMA
    for c in convs[:3]:
        w = P.unpack_conv_weight(c)
        assert ((P.unpack_split_weight(c) - w).abs().max() / w.abs().max()).item() < 1e-6
    # fp16 programs carry none
    assert all(c.sw is None for c in P.build_program("resnet18", dtype="fp16").all_convs())


# ---------------------------------------------------------------------------
# GPU: kernels against the fp64 oracle
# ---------------------------------------------------------------------------

@pytest.fixture(scope="module")
def ops():
    from idunno import ops as o

    o.load()
    return o


def _ref64(x_nhwc, w, b, stride, pad, relu, res=None):
    x = x_nhwc.double().permute(0, 3, 1, 2)
    y = F.conv2d(x, w.double().to(x.device), b.double().to(x.device), stride, pad)
    if res is not None:
        y = y + res.double().permute(0, 3, 1, 2)
    if relu:
        y = F.relu(y)
    return y.permute(0, 2, 3, 1)


def _check(y, ref, rel=2e-5):
    y = y.double()
    scale = ref.abs().max().item() + 1e-12
    err = (y - ref).abs().max().item()
    assert err <= rel * scale, f"max err {err:.3e} vs scale {scale:.3e} (rel {err / scale:.2e})"


SPLIT_CASES = [
    # (B, H, Cin, Cout, k, stride, pad)
    (2, 56, 64, 64, 3, 1, 1),      # resnet layer1
    (2, 56, 64, 128, 3, 2, 1),     # layer2 first conv
    (2, 56, 64, 128, 1, 2, 0),     # layer2 downsample
    (2, 28, 128, 128, 3, 1, 1),
    (2, 14, 256, 256, 3, 1, 1),
    (3, 7, 512, 512, 3, 1, 1),     # layer4, M = 147 (not a tile multiple)
    (2, 27, 64, 192, 5, 1, 2),     # alexnet conv2 (Cout 192 masks part of a tile)
    (2, 56, 256, 64, 1, 1, 0),     # resnet50 1x1 reduce
    (2, 14, 1024, 256, 1, 1, 0),
    (1, 9, 96, 32, 3, 1, 1),       # odd: C 96 (3 split stages), Cout 32
]


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,Cin,Cout,k,s,p", SPLIT_CASES)
def test_conv_split_default_tile(ops, B, H, Cin, Cout, k, s, p):
    torch.manual_seed(B * 1000 + H + Cin + Cout + k)
    x = torch.randn(B, H, H, Cin, device=DEV)
    w = torch.randn(Cout, Cin, k, k) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout) * 0.1
    sw, scale = P.pack_split_weight(w)
    y = ops.conv2d_split(ops.split_from_f32(x), sw.to(DEV), b.to(DEV), scale, k, k, s, p, True)
    assert y.dtype == torch.float16 and y.shape[-1] == 2 * Cout
    ref = _ref64(x, w, b, s, p, True)
    _check(P.from_split(y), ref)


# streaming split 1x1 conv (tile 80, conv1x1_stream.hip SPLIT): ResNet50 bottleneck
# and downsample shapes, partial last tiles, multi-slab Cout
@pytest.mark.gpu
@pytest.mark.parametrize("B,H,Cin,Cout,s,res", [
    (2, 56, 64, 256, 1, True), (2, 56, 64, 64, 1, False), (3, 28, 128, 512, 1, True), (2, 14, 256, 1024, 1, True),
    (2, 56, 256, 64, 1, False), (1, 13, 256, 384, 1, False), (2, 28, 512, 128, 1, False), (2, 7, 512, 2048, 1, True),
    (2, 56, 64, 128, 2, False), (2, 28, 256, 512, 2, False), (3, 14, 512, 1024, 2, False), (1, 9, 128, 256, 2, True)])
def test_conv_split_1x1_stream(ops, B, H, Cin, Cout, s, res):
    torch.manual_seed(B * 100 + H + Cin + Cout + s + res)
    x = torch.randn(B, H, H, Cin, device=DEV)
    w = torch.randn(Cout, Cin, 1, 1) / Cin ** 0.5
    b = torch.randn(Cout) * 0.1
    ho = (H - 1) // s + 1
    r = torch.randn(B, ho, ho, Cout, device=DEV) if res else None
    sw, scale = P.pack_split_weight(w)
    for relu in (True, False):
        y = ops.conv2d_split(ops.split_from_f32(x), sw.to(DEV), b.to(DEV), scale, 1, 1, s, 0, relu,
                             residual=None if r is None else ops.split_from_f32(r), tile=80)
        assert y.shape == (B, ho, ho, 2 * Cout)
        _check(P.from_split(y), _ref64(x, w, b, s, 0, relu, r))


@pytest.mark.gpu
@pytest.mark.parametrize("B,Ho,K1,K2,Cout,s", [(2, 56, 64, 64, 256, 1), (3, 28, 128, 256, 512, 2), (1, 9, 64, 64, 128, 1),
                                               (2, 13, 128, 256, 64, 2)])
def test_conv1x1_dual_split(ops, B, Ho, K1, K2, Cout, s):
    """Split bottleneck tail: expansion 1x1 + (strided) 1x1 downsample as one GEMM, vs fp64."""
    torch.manual_seed(B + Ho + K1 + K2 + Cout + s)
    H = (Ho - 1) * s + 1 + (s - 1)
    y = torch.randn(B, Ho, Ho, K1, device=DEV)
    x = torch.randn(B, H, H, K2, device=DEV)
    w3 = torch.randn(Cout, K1, 1, 1) / K1 ** 0.5
    wd = torch.randn(Cout, K2, 1, 1) / K2 ** 0.5 * 0.1       # different magnitudes: one shared scale
    b3, bd = torch.randn(Cout) * 0.1, torch.randn(Cout) * 0.1
    sw, scale = P.pack_split_weight(torch.cat([w3, wd], 1))
    out = ops.conv1x1_dual_split(ops.split_from_f32(y), ops.split_from_f32(x), sw.to(DEV), (b3 + bd).to(DEV),
                                 scale, s, True)
    assert out.shape == (B, Ho, Ho, 2 * Cout)
    ref = torch.relu(_ref64(y, w3, b3, 1, 0, False) + _ref64(x, wd, bd, s, 0, False))
    _check(P.from_split(out), ref)


@pytest.mark.gpu
def test_resnet50_split_fused_downsample_matches_unfused(ops):
    from idunno.models import HipRunner, build_program

    prog = build_program("resnet50", seed=0, randomize_bn=True, dtype="fp32")
    img = ops.synth_images(11, 0, 4, torch.device(DEV))
    outs = {}
    for fuse in (False, True):
        r = HipRunner(prog, DEV)
        r.fuse_down_1x1 = fuse
        outs[fuse] = r.logits(img).double()
    scale = outs[False].abs().max().item()
    assert (outs[True] - outs[False]).abs().max().item() <= 2e-5 * scale


SPLIT_TILES = [26, 27, 34, 36, 38, 42]


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,W", [(2, 56, 56), (3, 13, 49), (1, 9, 52), (160, 56, 56), (40, 56, 56),
                                   (150, 13, 52)])
@pytest.mark.parametrize("res", [False, True])
def test_conv_split_c64_rows(ops, B, H, W, res):
    """Row-streaming register-weight 3x3 64->64 kernel (tile 50, 16 couts per wave).
    Small batches run one-row bands (every row's tail fragment alone); B = 160 / 40
    at H = 56 run bands of 8 / 2 rows (tails of row pairs); B = 150 at H = 13 runs
    two-row bands whose last band has one row."""
    _c64_rows_case(ops, B, H, W, res)


def _c64_rows_case(ops, B, H, W, res):
    torch.manual_seed(B * H + W + res)
    x = torch.randn(B, H, W, 64, device=DEV)
    w = torch.randn(64, 64, 3, 3) / 24
    b = torch.randn(64) * 0.1
    r = torch.randn(B, H, W, 64, device=DEV) if res else None
    sw, scale = P.pack_split_weight(w)
    y = ops.conv2d_split(ops.split_from_f32(x), sw.to(DEV), b.to(DEV), scale, 3, 3, 1, 1, True,
                         residual=None if r is None else ops.split_from_f32(r), tile=50)
    _check(P.from_split(y), _ref64(x, w, b, 1, 1, True, r))


@pytest.mark.gpu
@pytest.mark.parametrize("tile", SPLIT_TILES)
@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("out_f32", [False, True])
def test_conv_split_tiles(ops, tile, res, out_f32):
    torch.manual_seed(tile + 7 * res + 3 * out_f32)
    B, H, Cin, Cout = 3, 13, 128, 192            # M = 507, Cout 192: partial tiles on both sides
    x = torch.randn(B, H, H, Cin, device=DEV)
    w = torch.randn(Cout, Cin, 3, 3) / (Cin * 9) ** 0.5
    b = torch.randn(Cout) * 0.1
    r = torch.randn(B, H, H, Cout, device=DEV) if res else None
    sw, scale = P.pack_split_weight(w)
    y = ops.conv2d_split(ops.split_from_f32(x), sw.to(DEV), b.to(DEV), scale, 3, 3, 1, 1, True,
                         residual=None if r is None else ops.split_from_f32(r), out_f32=out_f32, tile=tile)
    ref = _ref64(x, w, b, 1, 1, True, r)
    _check(y if out_f32 else P.from_split(y), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,cin,cout,k,s,ks", [(2, 9, 128, 256, 3, 1, 2), (2, 9, 128, 256, 3, 1, 3),
                                               (3, 7, 256, 512, 3, 1, 8), (2, 13, 64, 128, 3, 2, 6),
                                               (2, 14, 256, 512, 1, 2, 4), (1, 7, 512, 512, 3, 1, -1)])
@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("out_f32", [False, True])
def test_conv_split_ksplit(ops, B, H, cin, cout, k, s, ks, res, out_f32):
    """Small-M split-K (K slices of whole stage runs into fp32 partials, one
    combine with bias / residual / ReLU / re-split): forced k slices (k = 8 over
    72 stages starts slices inside a tap) and the auto pick (-1) at M = 49."""
    torch.manual_seed(B + H + cin + ks)
    x = torch.randn(B, H, H, cin, device=DEV)
    w = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
    b = torch.randn(cout) * 0.1
    pad = k // 2
    ho = (H + 2 * pad - k) // s + 1
    r = torch.randn(B, ho, ho, cout, device=DEV) if res else None
    sw, scale = P.pack_split_weight(w)
    y = ops.conv2d_split(ops.split_from_f32(x), sw.to(DEV), b.to(DEV), scale, k, k, s, pad, True,
                         residual=None if r is None else ops.split_from_f32(r), out_f32=out_f32, ksplit=ks)
    _check(y if out_f32 else P.from_split(y), _ref64(x, w, b, s, pad, True, r))


@pytest.mark.gpu
@pytest.mark.parametrize("kh,stride,pad,B", [(7, 2, 3, 3), (11, 4, 2, 2)])
@pytest.mark.parametrize("tile", [-1, 23, 27, 33, 35, 37])
def test_stem_pack3_split(ops, kh, stride, pad, B, tile):
    from idunno.models import reference as ref

    torch.manual_seed(kh + tile)
    img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=DEV)
    w = torch.randn(64, 3, kh, kh) / (3 * kh * kh) ** 0.5
    b = torch.randn(64) * 0.1
    sp3, scale = P.pack_split_weight_p3(w)
    x3 = ops.preprocess_pack3_split(img, kh, stride, pad)
    y = ops.conv2d_pack3_split(x3, sp3.to(DEV), b.to(DEV), scale, 224, kh, kh, stride, pad, True, tile=tile)
    assert y.dtype == torch.float32
    x = ref.preprocess_u8(img).permute(0, 2, 3, 1)
    _check(y, _ref64(x, w, b, stride, pad, True))


@pytest.mark.gpu
@pytest.mark.parametrize("B,hw", [(3, 224), (2, 100), (1, 37)])
def test_stem_split_fused(ops, B, hw):
    """uint8 -> normalise -> conv7x7/2 -> +bias -> ReLU -> maxpool3x3/2, split out
    (one cout fragment per wave, two conv rows per pass)."""
    from idunno.models import reference as ref

    torch.manual_seed(B + hw)
    img = torch.randint(0, 256, (B, hw, hw, 3), dtype=torch.uint8, device=DEV)
    w = torch.randn(64, 3, 7, 7) / (3 * 49) ** 0.5
    b = torch.randn(64) * 0.1
    fs, scale, bias, psum = P.pack_stem_split(w, b)
    y = ops.stem_split(img, fs.to(DEV), bias.to(DEV), psum.to(DEV), scale)
    x = ref.preprocess_u8(img).permute(0, 2, 3, 1)
    want = _ref64(x, w, b, 2, 3, True).permute(0, 3, 1, 2)
    want = F.max_pool2d(want, 3, 2, 1).permute(0, 2, 3, 1)
    assert y.shape == (*want.shape[:3], 128)
    _check(P.from_split(y), want)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 64])
@pytest.mark.parametrize("B,H,W", [(3, 224, 224), (2, 100, 131), (1, 31, 23), (5, 64, 72)])
def test_alex_stem_split_fused(ops, B, H, W, variant):
    """uint8 -> normalise -> conv11x11/4 pad 2 -> +bias -> ReLU -> maxpool3x3/2, split
    out, in one kernel (alex_stem.hip); ragged tiles and image borders included.
    variant: the kernel form (set_astem_variant; 0 one half per CU, 64 phased halves)."""
    from idunno.models import reference as ref

    ops.load().set_astem_variant(variant)
    try:
        _alex_stem_check(ops, B, H, W)
    finally:
        ops.load().set_astem_variant(64)


def _alex_stem_check(ops, B, H, W):
    from idunno.models import reference as ref

    torch.manual_seed(B + H)
    img = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=DEV)
    w = torch.randn(64, 3, 11, 11) / (3 * 121) ** 0.5
    b = torch.randn(64) * 0.1
    fs, scale, bias, psum = P.pack_alex_stem_split(w, b)
    y = ops.alex_stem_split(img, fs.to(DEV), bias.to(DEV), psum.to(DEV), scale)
    x = ref.preprocess_u8(img).permute(0, 2, 3, 1)
    want = _ref64(x, w, b, 4, 2, True).permute(0, 3, 1, 2)
    want = F.max_pool2d(want, 3, 2, 0).permute(0, 2, 3, 1)
    assert y.shape == (*want.shape[:3], 128)
    _check(P.from_split(y), want)
    # device-side window of an HBM-resident shard: rows start - offset .. + batch
    big = torch.cat([img, img.flip(0)])
    start = torch.tensor([B + 5], dtype=torch.long, device=DEV)
    y2 = ops.alex_stem_split(big, fs.to(DEV), bias.to(DEV), psum.to(DEV), scale, start, B, 5)
    assert torch.equal(y2, ops.alex_stem_split(img.flip(0).contiguous(), fs.to(DEV), bias.to(DEV),
                                               psum.to(DEV), scale))


@pytest.mark.gpu
def test_split_conversions_and_maxpool(ops):
    torch.manual_seed(5)
    x = torch.randn(3, 17, 19, 96, device=DEV) * 5
    xs = ops.split_from_f32(x)
    assert torch.equal(xs.cpu(), P.to_split(x.cpu()))
    back = ops.f32_from_split(xs)
    assert torch.equal(back.cpu(), P.from_split(xs.cpu()))
    ref = F.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    for inp in (x, xs):
        y = ops.maxpool2d_split(inp, 3, 2, 1)
        assert y.shape == (3, 9, 10, 192)
        _check(P.from_split(y.cpu()).to(DEV), ref.double(), rel=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,N,out_f32,relu,splits", [
    (500, 9216, 4096, False, True, None),    # alexnet fc6 (auto split)
    (500, 4096, 1000, True, False, None),    # fc8: N 1000, fp32 logits
    (7, 512, 96, False, False, 1),
    (33, 1024, 256, True, True, 4),
])
def test_linear_split(ops, M, K, N, out_f32, relu, splits):
    torch.manual_seed(M + K + N)
    x = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K) / K ** 0.5
    b = torch.randn(N) * 0.1
    sw, scale = P.pack_split_weight(w.reshape(N, K, 1, 1))
    y = ops.linear_split(ops.split_from_f32(x), sw.to(DEV), b.to(DEV), scale, relu=relu, out_f32=out_f32,
                         splits=splits)
    ref = x.double() @ w.double().t().to(DEV) + b.double().to(DEV)
    if relu:
        ref = F.relu(ref)
    _check(y if out_f32 else P.from_split(y), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name,B", [("resnet18", 4), ("resnet18", 400), ("resnet50", 8), ("alexnet", 6),
                                    ("alexnet", 500)])
def test_model_split_vs_fp64_oracle(ops, name, B):
    from idunno.models import reference as ref

    m = ref.build(name, seed=0)
    prog = P.compile_model(m, name, "fp32")
    r = P.HipRunner(prog)
    assert r.split and r._split_ok()
    img = ops.synth_images(0, 0, B, DEV)
    got = r.logits(img).double().cpu()
    if name.startswith("resnet") and B >= 8:
        # stem + layer1 on batch parts: the same numbers, up to the summation order of
        # a part's small-M 1x1 convs (M < 16384 runs them on the 128 x 64 tile, not
        # the streaming 1x1 kernel: conv1x1_small_m)
        r.split_front = 2
        got_f = r.logits(img).double().cpu()
        assert (got_f - got).abs().max().item() <= 2e-6 * got.abs().max().item()
        r.split_front = None
    if name.startswith("resnet") and B >= 64:
        # two half-batch streams: the same numbers, up to the summation order of
        # the small-M split-K (a half batch's layer4 runs as K slices)
        r.split_streams = 2
        got2 = r.logits(img).double().cpu()
        assert (got2 - got).abs().max().item() <= 2e-6 * got.abs().max().item()
        torch.cuda.synchronize()
        r.split_streams = None
    n = min(B, 8)
    with torch.no_grad():
        want = m.double()(ref.preprocess_u8(img[:n].cpu()).double())
    scale = want.abs().max().item()
    err = (got[:n] - want).abs().max().item() / scale
    assert err <= 1e-5, f"{name}: rel logit err {err:.2e}"
    assert torch.equal(got[:n].argmax(1), want.argmax(1))


# ---------------------------------------------------------------------------
# fp32 range on the split path: a value past 65504 has no
# finite fp16 hi half.  The split kernels flag it, softmax_top1 marks the batch
# class -2 and the runner / executor rerun it on the all-f32 kernels.
# ---------------------------------------------------------------------------

@pytest.mark.gpu
def test_split_guard_flags_residual_sum_past_fp16_range(ops):
    torch.manual_seed(5)
    x = P.to_split(torch.rand(2, 7, 7, 128, device=DEV) * 0.1)
    sw, scale = P.pack_split_weight(torch.randn(128, 128, 3, 3) * 0.01)
    sw = sw.to(DEV)
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)

    def run(bias, res):
        flag.zero_()
        ops.set_split_guard(flag)
        try:
            y = ops.conv2d_split(x, sw, torch.full((128,), bias, device=DEV), scale, 3, 3, 1, 1, False,
                                 residual=P.to_split(torch.full((2, 7, 7, 128), res, device=DEV)))
        finally:
            ops.set_split_guard(None)
        torch.cuda.synchronize()
        return int(flag.item()), y

    f, y = run(20000.0, 40000.0)               # every part and the sum < 65504
    assert f == 0 and bool(torch.isfinite(P.from_split(y)).all())
    f, _ = run(10000.0, 60000.0)               # each part fits, the sum does not
    assert f == 1
    f, _ = run(10000.0, 40000.0)               # the flag was reset: clean again
    assert f == 0


@pytest.mark.gpu
def test_split_activations_past_fp16_range_match_fp64(ops):
    """Stem weights x 1e5: activations ~1e5-1e6 and residual sums far past
    65504.  The split forward trips the guard and is recomputed on the f32
    kernels: logits match the fp64 oracle at the fp32 tolerance."""
    from idunno.models import reference as ref
    from idunno.runtime.executor import HipExecutor

    m = ref.build("resnet18", seed=3)
    with torch.no_grad():
        m.conv1.weight *= 1e5
    prog = P.compile_model(m, "resnet18", "fp32")
    r = P.HipRunner(prog)
    assert r.split and r._split_ok()
    img = ops.synth_images(4, 0, 4, DEV)
    with torch.no_grad():
        want = m.double()(ref.preprocess_u8(img.cpu()).double())
        act = torch.relu(m.bn1(m.conv1(ref.preprocess_u8(img.cpu()).double())))
    assert act.abs().max().item() > 1e5                               # the regime under test
    got = r.logits(img).double().cpu()
    assert r.overflow_reruns == 1
    scale = want.abs().max().item()
    err = (got - want).abs().max().item() / scale
    assert err <= 2e-5, f"rel logit err {err:.2e}"
    assert torch.equal(got.argmax(1), want.argmax(1))
    # the eager forward() classifies the rerun logits: no OVERFLOW_CLASS rows,
    # one f32 rerun per call (the stale flag marked every row -2)
    cls, prob = r.forward(img)
    assert r.overflow_reruns == 2
    assert torch.equal(cls.cpu().long(), want.argmax(1))
    assert abs(float(prob[0]) - torch.softmax(want, 1).max(1).values[0].item()) < 1e-4
    # a captured graph marks the batch instead (no host read inside the graph) ...
    sin, replay = r.capture(4)
    sin.copy_(img)
    cls, _ = replay()
    assert bool((cls == ops.OVERFLOW_CLASS).all())
    # ... and the executor reruns such a chunk on the f32 kernels
    ex = HipExecutor(DEV, seed=3)
    ex.runners["resnet18"] = r
    c2, p2 = ex.run("resnet18", img, 0, 3)
    assert (c2 == want.argmax(1).numpy()).all()
    assert abs(float(p2[0]) - torch.softmax(want, 1).max(1).values[0].item()) < 1e-4


# ---------------------------------------------------------------------------
# dual conv: a stride-2 block's 1x1/2 downsample in the launch of its 3x3/2
# conv (the downsample is the centre tap), halves read in place downstream
# ---------------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("B,H,C,Cout,tile", [(2, 56, 64, 128, -1), (3, 28, 128, 256, -1), (2, 14, 256, 512, -1),
                                             (3, 13, 64, 128, 36), (2, 9, 128, 256, 42), (1, 15, 64, 128, 34)])
def test_conv_split_dual_downsample(ops, B, H, C, Cout, tile):
    torch.manual_seed(B + H + C)
    x = torch.randn(B, H, H, C, device=DEV)
    w3 = torch.randn(Cout, C, 3, 3) / (9 * C) ** 0.5
    w1 = torch.randn(Cout, C, 1, 1) / C ** 0.5 * 3.0          # a different weight scale (own acc_scale2)
    b3, b1 = torch.randn(Cout) * 0.1, torch.randn(Cout) * 0.1
    s3, sc3 = P.pack_split_weight(w3)
    s1, sc1 = P.pack_split_weight(w1)
    c2 = s3.shape[1] // 9
    wd = torch.zeros(2 * Cout, s3.shape[1], dtype=s3.dtype)
    wd[:Cout] = s3
    wd[Cout:, 4 * c2:5 * c2] = s1
    xs = ops.split_from_f32(x)
    both = ops.conv2d_split_dual(xs, wd.to(DEV), torch.cat([b3, b1]).to(DEV), sc3, sc1, Cout, 3, 3, 2, 1, True,
                                 tile=tile)
    main, down = both[..., :2 * Cout], both[..., 2 * Cout:]
    _check(P.from_split(main.contiguous()), _ref64(x, w3, b3, 2, 1, True))
    _check(P.from_split(down.contiguous()), _ref64(x, w1, b1, 2, 0, False))
    # the next conv reads the halves in place: x with a 2x pixel stride, residual likewise
    w2 = torch.randn(Cout, Cout, 3, 3) / (9 * Cout) ** 0.5
    b2 = torch.randn(Cout) * 0.1
    s2, sc2 = P.pack_split_weight(w2)
    y = ops.conv2d_split(main, s2.to(DEV), b2.to(DEV), sc2, 3, 3, 1, 1, True, residual=down)
    y_ref = ops.conv2d_split(main.contiguous(), s2.to(DEV), b2.to(DEV), sc2, 3, 3, 1, 1, True,
                             residual=down.contiguous())
    assert torch.equal(y, y_ref)
    mid = P.from_split(main.contiguous()).double()
    _check(P.from_split(y), _ref64(mid, w2, b2, 1, 1, True, P.from_split(down.contiguous())))


@pytest.mark.gpu
def test_resnet18_fused_downsample_same_logits(ops):
    from idunno.models import reference as ref

    m = ref.build("resnet18", seed=2, randomize_bn=True)
    r = P.HipRunner(P.compile_model(m, "resnet18", "fp32"))
    img = ops.synth_images(7, 0, 24, DEV)
    r.fuse_down = True
    assert all(r._dual_ok(b) for b in r.p.blocks if b.down is not None)
    fused = r.logits(img).double()
    r.fuse_down = False
    plain = r.logits(img).double()
    scale = plain.abs().max().item()
    assert (fused - plain).abs().max().item() <= 1e-6 * scale
