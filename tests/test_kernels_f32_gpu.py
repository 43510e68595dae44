"""Reference-precision (fp32) path: every fp32 HIP kernel against plain PyTorch.

The oracle is F.conv2d & friends in float64 on the same fp32 inputs, so the
only difference the tests allow is fp32 rounding / summation order (the f32
MFMA is an exact-product fmaf chain).  Whole models are compared against the
fp64 CPU module on identical weights: max |logit error| / max |logit| <= 1e-4
("Next round" item 3).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    from idunno import ops as o

    o.load()
    return o


def _ref_conv64(x_nhwc, w, b, stride, pad, relu, res=None):
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


CONV_CASES = [
    # (B, H, Cin, Cout, k, stride, pad)
    (2, 56, 64, 64, 3, 1, 1),      # resnet layer1
    (2, 56, 64, 128, 3, 2, 1),     # layer2 first conv
    (2, 56, 64, 128, 1, 2, 0),     # layer2 downsample
    (2, 28, 128, 128, 3, 1, 1),
    (2, 14, 256, 256, 3, 1, 1),
    (3, 7, 512, 512, 3, 1, 1),     # layer4, M = 147 (not a tile multiple)
    (2, 27, 64, 192, 5, 1, 2),     # alexnet conv2 (Cout 192 masks part of a tile)
    (2, 13, 192, 384, 3, 1, 1),    # alexnet conv3
    (2, 56, 256, 64, 1, 1, 0),     # resnet50 1x1 reduce
    (2, 14, 1024, 256, 1, 1, 0),
    (1, 9, 48, 20, 3, 1, 1),       # odd: C 48 (3 BK=16 blocks), Cout 20
]


@pytest.mark.parametrize("B,H,Cin,Cout,k,s,p", CONV_CASES)
def test_conv_f32_default_tile(ops, B, H, Cin, Cout, k, s, p):
    from idunno.models.packed import pack_conv_weight

    torch.manual_seed(B * 1000 + H + Cin + Cout + k)
    x = torch.randn(B, H, H, Cin, device=DEV)
    w = torch.randn(Cout, Cin, k, k) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout) * 0.1
    pw, small = pack_conv_weight(w, "fp32")
    assert not small and pw.dtype == torch.float32
    y = ops.conv2d(x, pw.to(DEV), b.to(DEV), k, k, s, p, True)
    assert y.dtype == torch.float32
    ref = _ref_conv64(x, w, b, s, p, True)
    assert y.shape == ref.shape
    _check(y, ref)


F32_TILES = list(range(100, 110))


@pytest.mark.parametrize("tile", F32_TILES)
@pytest.mark.parametrize("H", [14, 9])
def test_conv_f32_all_tiles_with_residual(ops, tile, H):
    from idunno.models.packed import pack_conv_weight

    torch.manual_seed(tile * 31 + H)
    B, Cin, Cout = 2, 128, 256
    x = torch.randn(B, H, H, Cin, device=DEV)
    w = torch.randn(Cout, Cin, 3, 3) / (Cin * 9) ** 0.5
    b = torch.randn(Cout) * 0.1
    res = torch.randn(B, H, H, Cout, device=DEV)
    pw, _ = pack_conv_weight(w, "fp32")
    y = ops.conv2d(x, pw.to(DEV), b.to(DEV), 3, 3, 1, 1, True, residual=res, tile=tile)
    _check(y, _ref_conv64(x, w, b, 1, 1, True, res))


@pytest.mark.parametrize("tile", [t for t in F32_TILES if t != 101])
@pytest.mark.parametrize("B,H,k,s,p,Cout", [
    (2, 224, 7, 2, 3, 64),     # ResNet stem
    (2, 224, 11, 4, 2, 64),    # AlexNet conv1
    (1, 37, 7, 2, 3, 64),      # ragged image: padding taps on every border
    (3, 20, 5, 1, 2, 12),      # small Cout, tap blocks 2 (5 -> 8 taps)
])
def test_conv_f32_small_c_stems(ops, tile, B, H, k, s, p, Cout):
    """RGB stems on the small-C path: input NHWC4 from preprocess (4th channel
    zero), taps streamed as whole pixels, padding taps from the zero buffer."""
    from idunno.models.packed import pack_conv_weight
    from idunno.models.reference import preprocess_u8

    torch.manual_seed(H + k + tile)
    img = torch.randint(0, 256, (B, H, H, 3), dtype=torch.uint8, device=DEV)
    x4 = ops.preprocess(img, f32=True)
    w = torch.randn(Cout, 3, k, k) / (3 * k * k) ** 0.5
    b = torch.randn(Cout) * 0.1
    pw, small = pack_conv_weight(w, "fp32")
    assert small
    y = ops.conv2d(x4, pw.to(DEV), b.to(DEV), k, k, s, p, True, tile=tile)
    ref = _ref_conv64(preprocess_u8(img).permute(0, 2, 3, 1), w, b, s, p, True)
    _check(y, ref)


def test_preprocess_f32_matches_torchvision_math(ops):
    from idunno.models.reference import preprocess_u8

    torch.manual_seed(4)
    img = torch.randint(0, 256, (3, 224, 224, 3), dtype=torch.uint8, device=DEV)
    y = ops.preprocess(img, f32=True)
    assert y.dtype == torch.float32 and y.shape == (3, 224, 224, 4)
    ref = preprocess_u8(img).permute(0, 2, 3, 1)
    assert (y[..., :3] - ref).abs().max().item() < 1e-6
    assert y[..., 3].abs().max().item() == 0
    odd = torch.randint(0, 256, (3, 5, 7, 3), dtype=torch.uint8, device=DEV)
    yo = ops.preprocess(odd, f32=True)
    assert (yo[..., :3] - preprocess_u8(odd).permute(0, 2, 3, 1)).abs().max().item() < 1e-6


def test_pools_f32(ops):
    torch.manual_seed(3)
    x = torch.randn(3, 112, 112, 64, device=DEV)
    y = ops.maxpool2d(x, 3, 2, 1)
    assert y.dtype == torch.float32
    assert torch.equal(y, F.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1))
    x2 = torch.randn(2, 13, 13, 256, device=DEV)
    assert torch.equal(ops.maxpool2d(x2, 3, 2, 0), F.max_pool2d(x2.permute(0, 3, 1, 2), 3, 2, 0).permute(0, 2, 3, 1))
    for shape in [(4, 7, 7, 512), (2, 7, 7, 2048), (3, 5, 5, 12), (50, 7, 7, 512), (2, 3, 3, 1000), (1, 1, 1, 4)]:
        x3 = torch.randn(*shape, device=DEV)
        _check(ops.global_avgpool(x3), x3.double().mean(dim=(1, 2)), rel=1e-6)


@pytest.mark.parametrize("M,K,N,relu", [(400, 512, 1000, False), (7, 4096, 4096, True), (500, 9216, 256, True)])
def test_linear_f32(ops, M, K, N, relu):
    torch.manual_seed(M + K + N)
    x = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV) / K ** 0.5
    b = torch.randn(N, device=DEV) * 0.1
    y = ops.linear(x, w, b, relu=relu)
    ref = x.double() @ w.double().t() + b.double()
    if relu:
        ref = torch.relu(ref)
    _check(y, ref)


def _oracle(m, img, fp64):
    from idunno.models import reference as ref

    with torch.no_grad():
        if fp64:      # CPU float64 module
            return m.double().cpu()(ref.preprocess_u8(img.cpu()).double())
        return m.float().to(DEV)(ref.preprocess_u8(img)).double().cpu()   # plain PyTorch fp32 on the GPU


@pytest.mark.parametrize("name,B,fp64", [("resnet18", 8, True), ("alexnet", 4, True), ("resnet50", 4, True),
                                         ("resnet18", 400, False)])
def test_model_f32_vs_oracle(ops, name, B, fp64):
    """Whole fp32 program vs the module on identical (BN-randomised) weights
    (float64 on the CPU at small batch; PyTorch fp32 on the GPU at the bench's
    B = 400): max rel logit error <= 1e-4 and identical top-1 on every image
    whose oracle top-1/top-2 margin exceeds 1e-4 of the logit scale."""
    from idunno.models import HipRunner, compile_model
    from idunno.models import reference as ref

    m = ref.build(name, seed=7, randomize_bn=True)
    runner = HipRunner(compile_model(m, name, dtype="fp32"))
    g = torch.Generator(device=DEV).manual_seed(B + 1)
    img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=DEV, generator=g)
    logits = runner.logits(img).double().cpu()
    r = torch.cat([_oracle(m, img[i:i + 50], fp64) for i in range(0, B, 50)])
    scale = r.abs().max().item()
    err = (logits - r).abs().max().item()
    assert err <= 1e-4 * scale, f"{name}: rel logit err {err / scale:.2e}"
    cls, prob = runner.forward(img)
    top2 = r.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 1e-4 * scale
    assert torch.equal(cls.long().cpu()[clear], r.argmax(1)[clear])
    p_ref = torch.softmax(r, 1).gather(1, cls.long().cpu().view(-1, 1)).view(-1)
    assert (prob.double().cpu() - p_ref).abs().max().item() < 2e-5


def test_f32_window_graph_matches_eager(ops):
    """The bench path: hipGraph over a device-side window with packed output."""
    from idunno.models import HipRunner, build_program

    runner = HipRunner(build_program("resnet18", seed=5, dtype="fp32"))
    shard = ops.synth_images(99, 0, 40, "cuda")
    desc = torch.zeros(2, 4, dtype=torch.int64, device="cuda")
    packed = torch.full((8, 2), -1, dtype=torch.int32, device="cuda")
    _, run = runner.capture_window(shard, 8, start=desc[1, 2:3], packed=packed)
    for s0 in (0, 13, 35):         # 35 > 40 - 8: clamped to 32 on the device
        desc[1, 2] = s0
        c1, p1 = run()
        s = min(s0, 32)
        c0, p0 = runner.forward(shard[s:s + 8].contiguous())
        torch.cuda.synchronize()
        assert torch.equal(c0, c1) and torch.equal(p0, p1)
        assert torch.equal(packed[:, 0], c0)


WINO_CASES = [
    # (B, H, W, Cin, Cout)
    (2, 56, 56, 64, 64),      # resnet layer1: 2 tile rows per block, 14 blocks per image
    (2, 28, 28, 128, 128),    # layer2: partial last block (4, 4, 4, 2 tile rows)
    (2, 14, 14, 256, 256),    # layer3: one image per block (49 of 64 tile slots)
    (5, 7, 7, 512, 512),      # layer4: 4 images per block, odd size (padded 2x2 tiles), partial last block
    (2, 13, 13, 192, 384),    # alexnet conv3
    (1, 9, 5, 48, 32),        # odd everything
]


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("B,H,W,Cin,Cout", WINO_CASES)
def test_conv_wino_f32(ops, B, H, W, Cin, Cout, res, variant):
    """Fused Winograd F(2x2,3x3) fp32 conv vs the fp64 direct conv."""
    from idunno.models.packed import wino_weight

    torch.manual_seed(B + H * 7 + W + Cin + Cout + res)
    x = torch.randn(B, H, W, Cin, device=DEV)
    w = torch.randn(Cout, Cin, 3, 3) / (Cin * 9) ** 0.5
    b = torch.randn(Cout) * 0.1
    r = torch.randn(B, H, W, Cout, device=DEV) if res else None
    assert ops.wino_supported(H, W, Cin, Cout)
    y = ops.conv2d_wino(x, wino_weight(w).to(DEV), b.to(DEV), True, r, variant)
    _check(y, _ref_conv64(x, w, b, 1, 1, True, r), rel=5e-5)


@pytest.mark.parametrize("B,H,W,Cin,Cout", [
    (7, 14, 14, 32, 64),      # 49 tiles per image: blocks span up to 3 images
    (3, 28, 28, 32, 32),      # 196 tiles per image: blocks cross one image boundary
    (4, 13, 11, 16, 32),      # odd sizes: padded tiles inside consecutive-tile blocks
    (9, 7, 7, 16, 32),        # 16 tiles per image: the images-per-block mode
    (2, 56, 56, 16, 32),      # 28 tiles per row: LIN over 4-5 tile rows, 32-position rotated rows
])
def test_conv_wino_f32_linear(ops, B, H, W, Cin, Cout):
    """Variant 3 with its consecutive-tile (LIN) blocking (the rotated-raw-row and
    non-LIN A/B arms were folded away in round 5)."""
    from idunno.models.packed import wino_weight

    torch.manual_seed(B * H + W + Cin)
    x = torch.randn(B, H, W, Cin, device=DEV)
    w = torch.randn(Cout, Cin, 3, 3) / (Cin * 9) ** 0.5
    b = torch.randn(Cout) * 0.1
    r = torch.randn(B, H, W, Cout, device=DEV)
    y = ops.conv2d_wino(x, wino_weight(w).to(DEV), b.to(DEV), True, r, 3)
    _check(y, _ref_conv64(x, w, b, 1, 1, True, r), rel=5e-5)


def test_runner_winograd_matches_direct(ops):
    from idunno.models import HipRunner, build_program

    p = build_program("resnet18", seed=2, randomize_bn=True, dtype="fp32")
    img = ops.synth_images(5, 0, 6, DEV)
    a = HipRunner(p, winograd=True).logits(img)
    b = HipRunner(p, winograd=False).logits(img)
    assert (a - b).abs().max().item() <= 2e-5 * b.abs().max().item()


@pytest.mark.parametrize("tile", [-1] + [t for t in F32_TILES if t != 101])
@pytest.mark.parametrize("B,H,W,k,s,p,Cout", [
    (2, 224, 224, 7, 2, 3, 64),     # ResNet stem
    (2, 224, 224, 11, 4, 2, 64),    # AlexNet conv1
    (1, 37, 29, 7, 2, 3, 64),       # ragged image, odd width: both row copies, padding on every border
    (3, 20, 20, 5, 1, 2, 12),       # stride 1: four row copies
])
def test_conv_f32_pack3_stems(ops, tile, B, H, W, k, s, p, Cout):
    """RGB stems on packed rows (preprocess_pack3 + conv_f32 mode 2) vs fp64."""
    from idunno.models.packed import pack_conv_weight_p3
    from idunno.models.reference import preprocess_u8

    torch.manual_seed(H + k + tile)
    img = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=DEV)
    w = torch.randn(Cout, 3, k, k) / (3 * k * k) ** 0.5
    b = torch.randn(Cout) * 0.1
    x3 = ops.preprocess_pack3(img, k, s, p)
    y = ops.conv2d_pack3(x3, pack_conv_weight_p3(w).to(DEV), b.to(DEV), W, k, k, s, p, True, tile)
    ref = _ref_conv64(preprocess_u8(img).permute(0, 2, 3, 1), w, b, s, p, True)
    assert y.shape == ref.shape
    _check(y, ref)


def test_preprocess_pack3_window(ops):
    """Device-side window start (graph capture) reads the same images as slicing."""
    torch.manual_seed(11)
    shard = torch.randint(0, 256, (10, 32, 30, 3), dtype=torch.uint8, device=DEV)
    start = torch.tensor([103], dtype=torch.int64, device=DEV)        # global index, shard starts at 100
    a = ops.preprocess_pack3(shard, 7, 2, 3, start, 4, 100)
    b = ops.preprocess_pack3(shard[3:7].contiguous(), 7, 2, 3)
    assert torch.equal(a, b)
    part = ops.preprocess_pack3(shard, 7, 2, 3, start, 2, 100, 4, 2)
    assert torch.equal(part, b[2:])


@pytest.mark.parametrize("name", ["resnet18", "alexnet"])
def test_runner_pack3_matches_nhwc4_stem(ops, name):
    from idunno.models import HipRunner, build_program

    p = build_program(name, seed=3, randomize_bn=True, dtype="fp32")
    img = ops.synth_images(9, 0, 5, DEV)
    a = HipRunner(p, pack3=True).logits(img)
    b = HipRunner(p, pack3=False).logits(img)
    assert (a - b).abs().max().item() <= 2e-5 * b.abs().max().item()


@pytest.mark.parametrize("dtype", ["fp32", "fp16"])
def test_runner_side_stream_downsample(ops, dtype):
    """Downsample convs on a second stream (eager and captured) give the same logits."""
    from idunno.models import HipRunner, build_program

    p = build_program("resnet18", seed=5, randomize_bn=True, dtype=dtype)
    img = ops.synth_images(3, 0, 16, DEV)
    a = HipRunner(p)
    b = HipRunner(p)
    b.side_down = True
    la, lb = a.logits(img), b.logits(img)
    assert torch.equal(la, lb)
    sin, run = b.capture(16)
    sin.copy_(img)
    cls, prob = run()
    c0, p0 = a.forward(img)
    torch.cuda.synchronize()
    assert torch.equal(cls, c0) and torch.equal(prob, p0)


def test_runner_stem_parts_bitwise(ops):
    """fp32 stem + maxpool on batch parts (eager and device-window graph) = one pass."""
    from idunno.models import HipRunner, build_program

    p = build_program("resnet18", seed=6, randomize_bn=True, dtype="fp32")
    shard = ops.synth_images(4, 0, 24, DEV)
    a = HipRunner(p)
    b = HipRunner(p)
    b.stem_parts = 3
    assert torch.equal(a.logits(shard[:10]), b.logits(shard[:10]))
    _s, run_a = a.capture_window(shard, 12)
    _s2, run_b = b.capture_window(shard, 12)
    ca, pa = run_a()
    cb, pb = run_b()
    torch.cuda.synchronize()
    assert torch.equal(ca, cb) and torch.equal(pa, pb)


@pytest.mark.parametrize("splits", [1, 2, 4, 8])
@pytest.mark.parametrize("M,K,N", [(500, 9216, 4096), (37, 512, 1000), (130, 2048, 36)])
def test_linear_f32_splitk_one_launch(ops, M, K, N, splits):
    """fp32 FC with split-K slices in one conv_f32 launch + combine, vs fp64."""
    torch.manual_seed(M + K + N + splits)
    x = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV) / K ** 0.5
    b = torch.randn(N, device=DEV) * 0.1
    y = ops.load().linear_f32_splitk(x, w, b, True, splits, -1)
    _check(y, torch.relu(x.double() @ w.double().t() + b.double()))
