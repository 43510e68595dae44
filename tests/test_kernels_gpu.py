"""Numerics of every gfx950 HIP kernel against a plain PyTorch fp32 reference.

Shapes follow SURVEY.md §2.4 (ResNet18 / AlexNet / ResNet50 layer list) at a
small batch; inputs are random and asymmetric so a transposed store or a
swapped fragment map cannot pass.
"""
import os

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


def _ref_conv(x_nhwc, w, b, stride, pad, relu, res=None):
    x = x_nhwc.float().permute(0, 3, 1, 2)
    y = F.conv2d(x, w.float(), b.float(), stride, pad)
    if res is not None:
        y = y + res.float().permute(0, 3, 1, 2)
    if relu:
        y = F.relu(y)
    return y.permute(0, 2, 3, 1)


def _check(y, ref, tol=1e-2):
    y = y.float()
    scale = ref.abs().max().item() + 1e-6
    err = (y - ref).abs().max().item()
    assert err <= tol * scale + 1e-3, f"max err {err} vs scale {scale}"


CONV_CASES = [
    # (B, H, Cin, Cout, k, stride, pad)
    (2, 56, 64, 64, 3, 1, 1),      # resnet layer1
    (2, 56, 64, 128, 3, 2, 1),     # layer2 first conv
    (2, 56, 64, 128, 1, 2, 0),     # layer2 downsample
    (2, 28, 128, 128, 3, 1, 1),
    (2, 14, 256, 256, 3, 1, 1),
    (3, 7, 512, 512, 3, 1, 1),     # layer4, M = 147 (not a tile multiple)
    (2, 27, 64, 192, 5, 1, 2),     # alexnet conv2
    (2, 13, 192, 384, 3, 1, 1),    # alexnet conv3
    (2, 56, 256, 64, 1, 1, 0),     # resnet50 1x1 reduce
    (2, 14, 1024, 256, 1, 1, 0),
]


@pytest.mark.parametrize("B,H,Cin,Cout,k,s,p", CONV_CASES)
def test_conv_shapes(ops, B, H, Cin, Cout, k, s, p):
    from idunno.models.packed import pack_conv_weight

    torch.manual_seed(B * 1000 + H + Cin + Cout + k)
    x = torch.randn(B, H, H, Cin, device=DEV).half()
    w = (torch.randn(Cout, Cin, k, k) / (Cin * k * k) ** 0.5)
    b = torch.randn(Cout) * 0.1
    pw, small = pack_conv_weight(w)
    assert not small
    wq = w.half().float()
    y = ops.conv2d(x, pw.to(DEV), b.to(DEV), k, k, s, p, True)
    ref = _ref_conv(x, wq.to(DEV), b.to(DEV), s, p, True)
    assert y.shape == ref.shape
    _check(y, ref)


@pytest.mark.parametrize("B,H,cin,cout,k,s,ks", [(2, 9, 128, 256, 3, 1, 2), (2, 9, 128, 256, 3, 1, 3),
                                               (3, 7, 512, 512, 3, 1, 8), (2, 13, 128, 128, 3, 2, 6),
                                               (2, 14, 256, 512, 1, 2, 4), (1, 7, 512, 512, 3, 1, -1)])
@pytest.mark.parametrize("res", [False, True])
def test_conv_f16_ksplit(ops, B, H, cin, cout, k, s, ks, res):
    """fp16 convs at small M as K slices + one combine (forced slice counts; -1:
    the auto pick at M = 49) against the fp32 reference."""
    from idunno.models.packed import pack_conv_weight

    torch.manual_seed(B + H + cin + ks + res)
    x = torch.randn(B, H, H, cin, device=DEV).half()
    w = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
    b = torch.randn(cout) * 0.1
    pad = k // 2
    ho = (H + 2 * pad - k) // s + 1
    r = torch.randn(B, ho, ho, cout, device=DEV).half() if res else None
    pw, small = pack_conv_weight(w)
    y = ops.conv2d(x, pw.to(DEV), b.to(DEV), k, k, s, pad, True, residual=r, ksplit=ks)
    _check(y, _ref_conv(x, w.half().float().to(DEV), b.to(DEV), s, pad, True, r))


@pytest.mark.parametrize("tile", [0, 1, 2, 3] + list(range(10, 40)) + [42])
@pytest.mark.parametrize("H", [14, 9])
def test_conv_all_tiles_with_residual(ops, tile, H):
    from idunno.models.packed import pack_conv_weight

    torch.manual_seed(tile * 31 + H)
    B, Cin, Cout = 2, 128, 256 if tile == 17 else 128
    x = torch.randn(B, H, H, Cin, device=DEV).half()
    w = torch.randn(Cout, Cin, 3, 3) / (Cin * 9) ** 0.5
    b = torch.randn(Cout) * 0.1
    res = torch.randn(B, H, H, Cout, device=DEV).half()
    pw, _ = pack_conv_weight(w)
    y = ops.conv2d(x, pw.to(DEV), b.to(DEV), 3, 3, 1, 1, True, residual=res, tile=tile)
    ref = _ref_conv(x, w.half().float().to(DEV), b.to(DEV), 1, 1, True, res)
    _check(y, ref)


# streaming 1x1 conv (tile 80, conv1x1_stream.hip): the ResNet50 bottleneck 1x1
# shapes; M values that leave a partial last tile and give some workgroups one
# item, others several (B*H*H vs the 2-per-CU resident grid)
@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("B,H,Cin,Cout,res", [
    (3, 56, 64, 256, True), (3, 56, 64, 256, False), (2, 56, 64, 64, False), (5, 28, 128, 512, True),
    (1, 9, 64, 256, True), (1, 7, 128, 512, False), (2, 13, 64, 512, True), (40, 56, 64, 256, True),
    (2, 56, 256, 64, False), (3, 14, 256, 1024, True), (2, 20, 256, 128, False), (1, 11, 256, 384, True),
    (2, 28, 512, 128, False), (3, 7, 512, 2048, True)])
def test_conv1x1_stream(ops, B, H, Cin, Cout, res, stride):
    """Residual and output through per-wave LDS tiles where the shape allows (LIO), registers otherwise."""
    from idunno.models.packed import pack_conv_weight

    torch.manual_seed(B * 7 + H + Cin + Cout + res + stride)
    x = torch.randn(B, H, H, Cin, device=DEV).half()
    w = torch.randn(Cout, Cin, 1, 1) / Cin ** 0.5
    b = torch.randn(Cout) * 0.1
    ho = (H - 1) // stride + 1
    r = torch.randn(B, ho, ho, Cout, device=DEV).half() if res else None
    pw, _ = pack_conv_weight(w)
    for relu in (True, False):
        y = ops.conv2d(x, pw.to(DEV), b.to(DEV), 1, 1, stride, 0, relu, residual=r, tile=80)
        ref = _ref_conv(x, w.half().float().to(DEV), b.to(DEV), stride, 0, relu, r)
        _check(y, ref)
        # same rounding as the implicit-GEMM tile: identical fp16 outputs
        y36 = ops.conv2d(x, pw.to(DEV), b.to(DEV), 1, 1, stride, 0, relu, residual=r, tile=36)
        assert (y.float() - y36.float()).abs().max().item() <= 2e-3 * (y36.float().abs().max().item() + 1)


@pytest.mark.parametrize("B,Ho,K1,K2,Cout,s", [(2, 56, 64, 64, 256, 1), (3, 28, 128, 256, 512, 2), (1, 9, 64, 64, 512, 1),
                                               (2, 13, 128, 256, 128, 2)])
def test_conv1x1_dual(ops, B, Ho, K1, K2, Cout, s):
    """Bottleneck expansion 1x1 + 1x1 downsample as one GEMM over [y | x]."""
    from idunno.models.packed import pack_conv_weight

    torch.manual_seed(B + Ho + K1 + K2 + Cout + s)
    H = (Ho - 1) * s + 1 + (s - 1)
    y = torch.randn(B, Ho, Ho, K1, device=DEV).half()
    x = torch.randn(B, H, H, K2, device=DEV).half()
    w3 = torch.randn(Cout, K1, 1, 1) / K1 ** 0.5
    wd = torch.randn(Cout, K2, 1, 1) / K2 ** 0.5
    b3, bd = torch.randn(Cout) * 0.1, torch.randn(Cout) * 0.1
    p3, _ = pack_conv_weight(w3)
    pd, _ = pack_conv_weight(wd)
    w = torch.cat([p3, pd], 1).to(DEV).contiguous()
    out = ops.conv1x1_dual(y, x, w, (b3 + bd).to(DEV), s, True)
    ref = F.relu(_ref_conv(y, w3.half().float().to(DEV), b3.to(DEV), 1, 0, False)
                 + _ref_conv(x, wd.half().float().to(DEV), bd.to(DEV), s, 0, False))
    assert out.shape == ref.shape
    _check(out, ref)


@pytest.mark.parametrize("B,H,N2,dual", [(2, 56, 64, False), (3, 20, 128, False), (2, 56, 64, True), (1, 9, 64, True)])
def test_conv1x1_fused_next(ops, B, H, N2, dual):
    """Bottleneck tail (residual or dual form) + the next block's reduce 1x1 from the on-chip tile
    (residual, output and z through LDS tiles)."""
    from idunno.models.packed import pack_conv_weight

    torch.manual_seed(B + H + N2 + dual)
    y = torch.randn(B, H, H, 64, device=DEV).half()
    x = torch.randn(B, H, H, 64 if dual else 256, device=DEV).half()
    w3 = torch.randn(256, 64, 1, 1) / 8
    b3 = torch.randn(256) * 0.1
    w2 = torch.randn(N2, 256, 1, 1) / 16
    b2 = torch.randn(N2) * 0.1
    p3, _ = pack_conv_weight(w3)
    p2, _ = pack_conv_weight(w2)
    ext = ops.load()
    if dual:
        wd = torch.randn(256, 64, 1, 1) / 8
        bd = torch.randn(256) * 0.1
        pd, _ = pack_conv_weight(wd)
        wcat = torch.cat([p3, pd], 1).to(DEV).contiguous()
        run = lambda: ops.conv1x1_fused_next(y, wcat, (b3 + bd).to(DEV), p2.to(DEV), b2.to(DEV), x2=x)
        ref = F.relu(_ref_conv(y, w3.half().float().to(DEV), b3.to(DEV), 1, 0, False)
                     + _ref_conv(x, wd.half().float().to(DEV), bd.to(DEV), 1, 0, False))
    else:
        run = lambda: ops.conv1x1_fused_next(y, p3.to(DEV), b3.to(DEV), p2.to(DEV), b2.to(DEV), residual=x)
        ref = _ref_conv(y, w3.half().float().to(DEV), b3.to(DEV), 1, 0, True, x)
    out, z = run()
    _check(out, ref)
    # z is exactly the reduce conv of the stored (fp16) output
    z_ref = ops.conv2d(out, p2.to(DEV), b2.to(DEV), 1, 1, 1, 0, True, tile=36)
    assert (z.float() - z_ref.float()).abs().max().item() <= 2e-3 * (z_ref.float().abs().max().item() + 1)


def test_resnet50_fused_next_matches_unfused(ops):
    from idunno.models import HipRunner, build_program

    prog = build_program("resnet50", seed=0, randomize_bn=True)
    img = ops.synth_images(5, 0, 6, torch.device(DEV))
    outs = {}
    for fuse in (False, True):
        r = HipRunner(prog, DEV)
        r.fuse_next_1x1 = fuse
        outs[fuse] = r.logits(img).float()
    scale = outs[False].abs().max().item()
    assert (outs[True] - outs[False]).abs().max().item() <= 1e-2 * scale


def test_resnet50_fused_downsample_matches_unfused(ops):
    from idunno.models import HipRunner, build_program

    torch.manual_seed(0)
    prog = build_program("resnet50", seed=0, randomize_bn=True)
    img = ops.synth_images(7, 0, 6, torch.device(DEV))
    outs = {}
    for fuse in (False, True):
        r = HipRunner(prog, DEV)
        r.fuse_down_1x1 = fuse
        outs[fuse] = r.logits(img).float()
    scale = outs[False].abs().max().item()
    assert (outs[True] - outs[False]).abs().max().item() <= 2e-2 * scale
    # top-1 agrees wherever the unfused top-2 margin exceeds the fp16 noise (random
    # init nets have near ties; the fused GEMM rounds the residual sum once, not twice)
    top2 = outs[False].topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 2e-3 * scale
    assert torch.equal(outs[True].argmax(1)[clear], outs[False].argmax(1)[clear])




@pytest.mark.parametrize("k,s,p,H", [(7, 2, 3, 224), (11, 4, 2, 224), (7, 2, 3, 37)])
def test_conv_small_c_stem(ops, k, s, p, H):
    from idunno.models.packed import pack_conv_weight

    torch.manual_seed(k * 7 + H)
    B, Cout = 2, 64
    x3 = torch.randn(B, H, H, 3, device=DEV).half()
    x4 = torch.zeros(B, H, H, 4, device=DEV).half()
    x4[..., :3] = x3
    w = torch.randn(Cout, 3, k, k) / (3 * k * k) ** 0.5
    b = torch.randn(Cout) * 0.1
    pw, small = pack_conv_weight(w)
    assert small
    y = ops.conv2d(x4, pw.to(DEV), b.to(DEV), k, k, s, p, True)
    ref = _ref_conv(x3, w.half().float().to(DEV), b.to(DEV), s, p, True)
    _check(y, ref)


@pytest.mark.parametrize("B,K,N", [(5, 512, 1000), (7, 9216, 4096), (16, 2048, 1000)])
def test_linear_fp32_out(ops, B, K, N):
    torch.manual_seed(B + K + N)
    x = torch.randn(B, K, device=DEV).half()
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).half()
    b = torch.randn(N, device=DEV)
    y = ops.linear(x, w, b, relu=False, out_f32=True)
    assert y.dtype == torch.float32 and y.shape == (B, N)
    ref = x.float() @ w.float().t() + b
    _check(y, ref, tol=5e-3)


@pytest.mark.parametrize("splits", [1, 2, 4, 8])
@pytest.mark.parametrize("B,K,N,relu,f32", [(500, 9216, 4096, True, False), (500, 4096, 1000, False, True),
                                            (130, 2048, 1000, False, True)])
def test_linear_split_k(ops, B, K, N, relu, f32, splits):
    """FC through split-K partial GEMMs (K-slices of each row, ldx = K) + combine."""
    torch.manual_seed(B + K + N + (splits or 0))
    x = torch.randn(B, K, device=DEV).half()
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).half()
    b = torch.randn(N, device=DEV)
    y = ops.linear(x, w, b, relu=relu, out_f32=f32, splits=splits)
    assert y.dtype == (torch.float32 if f32 else torch.float16) and y.shape == (B, N)
    ref = x.float() @ w.float().t() + b
    if relu:
        ref = torch.relu(ref)
    _check(y, ref, tol=5e-3)


def test_maxpool_and_avgpool(ops):
    torch.manual_seed(3)
    x = torch.randn(3, 112, 112, 64, device=DEV).half()
    y = ops.maxpool2d(x, 3, 2, 1)
    ref = F.max_pool2d(x.float().permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.equal(y.float(), ref)
    x2 = torch.randn(2, 13, 13, 256, device=DEV).half()
    y2 = ops.maxpool2d(x2, 3, 2, 0)
    ref2 = F.max_pool2d(x2.float().permute(0, 3, 1, 2), 3, 2, 0).permute(0, 2, 3, 1)
    assert torch.equal(y2.float(), ref2)
    x3 = torch.randn(4, 7, 7, 512, device=DEV).half()
    a = ops.global_avgpool(x3)
    _check(a, x3.float().mean(dim=(1, 2)), tol=2e-3)


def test_preprocess_and_resize_crop(ops):
    from idunno.models.reference import preprocess_u8

    torch.manual_seed(4)
    img = torch.randint(0, 256, (2, 224, 224, 3), dtype=torch.uint8, device=DEV)
    y = ops.preprocess(img)
    ref = preprocess_u8(img).permute(0, 2, 3, 1)
    assert y.shape == (2, 224, 224, 4)
    assert (y[..., :3].float() - ref).abs().max().item() < 5e-3
    assert y[..., 3].abs().max().item() == 0
    # ragged pixel count (105 = 26 quads + 1) and a source 1 byte off alignment:
    # the per-byte fallback of the 4-pixel kernel
    for off in (0, 1):
        buf = torch.randint(0, 256, (off + 3 * 5 * 7 * 3,), dtype=torch.uint8, device=DEV)
        odd = buf[off:].view(3, 5, 7, 3)
        yo = ops.preprocess(odd)
        refo = preprocess_u8(odd).permute(0, 2, 3, 1)
        assert yo.shape == (3, 5, 7, 4)
        assert (yo[..., :3].float() - refo).abs().max().item() < 5e-3
        assert yo[..., 3].abs().max().item() == 0
    big = torch.randint(0, 256, (2, 300, 400, 3), dtype=torch.uint8, device=DEV)
    z = ops.resize_crop(big, 256, 224)
    assert z.shape == (2, 224, 224, 4)
    # reference: bilinear (align_corners=False, no antialias) + centre crop
    f = big.permute(0, 3, 1, 2).float()
    r = F.interpolate(f, size=(256, 341), mode="bilinear", align_corners=False)
    top, left = (256 - 224 + 1) // 2, (341 - 224 + 1) // 2
    r = r[:, :, top:top + 224, left:left + 224].clamp(0, 255)
    mean = torch.tensor([0.485, 0.456, 0.406], device=DEV).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], device=DEV).view(1, 3, 1, 1)
    r = ((r / 255 - mean) / std).permute(0, 2, 3, 1)
    assert (z[..., :3].float() - r).abs().max().item() < 2e-2


def test_softmax_top1(ops):
    torch.manual_seed(5)
    logits = torch.randn(37, 1000, device=DEV) * 3
    logits[3, 10] = logits[3, 20] = 100.0  # tie -> lowest index
    cls, prob = ops.softmax_top1(logits)
    p = torch.softmax(logits, dim=1)
    v, i = p.max(dim=1)
    assert torch.equal(cls.long(), i)
    assert cls[3].item() == 10
    assert torch.allclose(prob, v, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("N", [10, 64, 1000, 1024, 1500])
def test_softmax_top1_widths(ops, N):
    """Register-resident rows (N <= 1024) and the streaming fallback (N > 1024);
    ties inside one lane (j, j + 64) and across lanes resolve to the lowest index."""
    torch.manual_seed(N)
    logits = torch.randn(9, N, device=DEV)
    if N > 80:
        logits[1, 74] = logits[1, 10] = 50.0      # same lane (10 = 74 - 64)
        logits[2, N - 1] = logits[2, 3] = 50.0    # different lanes
    cls, prob = ops.softmax_top1(logits)
    p = torch.softmax(logits.double(), dim=1)
    v, i = p.max(dim=1)
    assert torch.equal(cls.long(), i)
    if N > 80:
        assert cls[1].item() == 10 and cls[2].item() == 3
    assert torch.allclose(prob.double(), v, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("name", ["resnet18", "alexnet", "resnet50"])
def test_model_end_to_end_vs_fp32_oracle(ops, name):
    from idunno.models import HipRunner, compile_model
    from idunno.models import reference as ref

    m = ref.build(name, seed=7, randomize_bn=True)
    prog = compile_model(m, name)
    runner = HipRunner(prog)
    torch.manual_seed(8)
    img = torch.randint(0, 256, (8, 224, 224, 3), dtype=torch.uint8, device=DEV)
    logits = runner.logits(img)
    with torch.no_grad():
        r = m.to(DEV)(ref.preprocess_u8(img))
    scale = r.abs().max().item()
    err = (logits - r).abs().max().item()
    assert err < 0.03 * scale, f"{name}: logits err {err} vs scale {scale}"
    cls, prob = runner.forward(img)
    agree = (cls.long() == r.argmax(1)).float().mean().item()
    assert agree >= 0.85, f"top-1 agreement {agree}"


@pytest.mark.parametrize("name,B", [("resnet18", 1), ("resnet18", 80), ("resnet18", 400), ("alexnet", 1),
                                    ("alexnet", 500), ("resnet50", 1024)])
def test_model_batch_sizes_vs_fp32_oracle(ops, name, B):
    """whole-model forward at B in {1, 80, 400, 1024} (and the
    AlexNet query size 500) against the fp32 PyTorch oracle on identical
    weights: logits within 3 % of their scale, and the same top-1 class on every
    image whose oracle top-1/top-2 margin exceeds 2 % of that scale."""
    from idunno.models import HipRunner, compile_model
    from idunno.models import reference as ref

    m = ref.build(name, seed=11, randomize_bn=True)
    runner = HipRunner(compile_model(m, name))
    g = torch.Generator(device=DEV).manual_seed(B)
    img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=DEV, generator=g)
    logits = runner.logits(img)
    with torch.no_grad():
        r = torch.cat([m.to(DEV)(ref.preprocess_u8(img[i:i + 128])) for i in range(0, B, 128)])
    scale = r.abs().max().item()
    assert (logits - r).abs().max().item() < 0.03 * scale
    cls, prob = runner.forward(img)
    top2 = r.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 0.02 * scale
    assert torch.equal(cls.long()[clear], r.argmax(1)[clear])
    p_ref = torch.softmax(r, 1).gather(1, cls.long().view(-1, 1)).view(-1)
    assert (prob - p_ref).abs().max().item() < 0.02


def test_hipgraph_replay_matches_eager(ops):
    from idunno.models import HipRunner, build_program

    runner = HipRunner(build_program("resnet18", seed=3))
    torch.manual_seed(9)
    img = torch.randint(0, 256, (16, 224, 224, 3), dtype=torch.uint8, device=DEV)
    c0, p0 = runner.forward(img)
    sin, run = runner.capture(16)
    sin.copy_(img)
    c1, p1 = run()
    torch.cuda.synchronize()
    assert torch.equal(c0, c1)
    assert torch.allclose(p0, p1)


def test_direct_graph_launch_matches_replay(ops):
    """IDUNNO_DIRECT_LAUNCH: the captured graph launched with hipGraphLaunch on
    the current stream (ops graph_launch) gives the torch replay's results."""
    from idunno.models import HipRunner, build_program

    shard = ops.synth_images(7, 0, 24, "cuda")
    outs = []
    for direct in (False, True):
        runner = HipRunner(build_program("resnet18", seed=4))
        runner.direct_launch = direct
        start, run = runner.capture_window(shard, 8)
        res = []
        for s0 in (0, 9, 16):
            start.fill_(s0)
            c, p = run()
            res.append((c.clone(), p.clone()))
        torch.cuda.synchronize()
        outs.append(res)
    for (c0, p0), (c1, p1) in zip(*outs):
        assert torch.equal(c0, c1) and torch.equal(p0, p1)


@pytest.mark.parametrize("fuse", [True, False])
def test_device_window_graph_matches_slices(ops, fuse):
    from idunno.models import HipRunner, build_program

    runner = HipRunner(build_program("resnet18", seed=5), fuse_stem=fuse)
    shard = ops.synth_images(99, 0, 40, "cuda")
    start, run = runner.capture_window(shard, 8)
    for s0 in (0, 13, 32, 35):     # 35 > 40 - 8: clamped to 32 on the device
        start.fill_(s0)
        c1, p1 = run()
        s = min(s0, 32)
        c0, p0 = runner.forward(shard[s:s + 8].contiguous())
        torch.cuda.synchronize()
        assert torch.equal(c0, c1) and torch.allclose(p0, p1)


@pytest.mark.parametrize("split", [2, 3])
def test_front_split_bit_identical(ops, split):
    """Stem + layer1 on batch parts (window parts through the device-side start)
    give exactly the unsplit results, eager and captured."""
    from idunno.models import HipRunner, build_program

    prog = build_program("resnet18", seed=4)
    one, many = HipRunner(prog, front_split=1), HipRunner(prog, front_split=split)
    shard = ops.synth_images(3, 0, 30, "cuda")
    c1, p1 = one.forward(shard[:10].contiguous())
    c2, p2 = many.forward(shard[:10].contiguous())
    assert torch.equal(c1, c2) and torch.equal(p1, p2)
    s1, r1 = one.capture_window(shard, 11)
    s2, r2 = many.capture_window(shard, 11)
    for s0 in (0, 5, 25):                      # 25 > 30 - 11: clamped to 19 for every part
        s1.fill_(s0)
        s2.fill_(s0)
        a, b = r1(), r2()
        torch.cuda.synchronize()
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("fuse", [True, False])
def test_window_from_descriptor_row_with_packed_output(ops, fuse):
    """Graph reads a GLOBAL start index in place (minus the shard's base) and
    writes (class, prob bits) pairs into a caller buffer (bench / data plane)."""
    from idunno.models import HipRunner, build_program

    runner = HipRunner(build_program("resnet18", seed=6), fuse_stem=fuse)
    base = 1000
    shard = ops.synth_images(7, base, 24, "cuda")
    desc = torch.zeros(2, 4, dtype=torch.int64, device="cuda")
    packed = torch.full((8, 2), -1, dtype=torch.int32, device="cuda")
    _, run = runner.capture_window(shard, 8, start=desc[1, 2:3], start_offset=base, packed=packed)
    for g0 in (1000, 1009, 1016):
        desc[1, 2] = g0
        c1, p1 = run()
        s = g0 - base
        c0, p0 = runner.forward(shard[s:s + 8].contiguous())
        torch.cuda.synchronize()
        assert torch.equal(c0, c1) and torch.allclose(p0, p1)
        assert torch.equal(packed[:, 0], c0) and torch.equal(packed[:, 1].view(torch.float32), p1)


@pytest.mark.parametrize("B,H", [(3, 224), (2, 64), (1, 100), (2, 37)])
def test_stem_fused_vs_fp32(ops, B, H):
    from idunno.models.packed import pack_conv_weight
    from idunno.models.reference import preprocess_u8

    torch.manual_seed(H + B)
    img = torch.randint(0, 256, (B, H, H, 3), dtype=torch.uint8, device=DEV)
    w = torch.randn(64, 3, 7, 7) / (3 * 49) ** 0.5
    b = torch.randn(64) * 0.1
    pw, small = pack_conv_weight(w)
    y = ops.stem_fused(img, pw.to(DEV), b.to(DEV))
    x = preprocess_u8(img)
    ref = F.max_pool2d(F.relu(F.conv2d(x, w.half().float().to(DEV), b.to(DEV), 2, 3)), 3, 2, 1)
    ref = ref.permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    _check(y, ref)


@pytest.mark.parametrize("B,H", [(3, 224), (2, 64), (1, 100), (2, 37)])
def test_stem_u8_f16_vs_fp32(ops, B, H):
    """fp16 exact-u8 stem (split stem kernel, hi MFMA only) vs the fp32 conv of the same image."""
    from idunno.models.packed import pack_stem_split
    from idunno.models.reference import preprocess_u8

    torch.manual_seed(H + B + 1)
    img = torch.randint(0, 256, (B, H, H, 3), dtype=torch.uint8, device=DEV)
    w = torch.randn(64, 3, 7, 7) / (3 * 49) ** 0.5
    b = torch.randn(64) * 0.1
    fs, scale, bias, psum = pack_stem_split(w.double(), b.double())
    y = ops.stem_u8_f16(img, fs.to(DEV), bias.to(DEV), psum.to(DEV), scale)
    x = preprocess_u8(img)
    ref = F.max_pool2d(F.relu(F.conv2d(x, w.to(DEV), b.to(DEV), 2, 3)), 3, 2, 1).permute(0, 2, 3, 1)
    assert y.dtype == torch.float16 and y.shape == ref.shape
    _check(y, ref)


@pytest.mark.parametrize("two_wg", [False, True])
@pytest.mark.parametrize("B,H,W", [(3, 224, 224), (2, 100, 131), (1, 31, 23)])
def test_alex_stem_u8_f16_vs_fp32(ops, B, H, W, two_wg):
    """fp16 fused AlexNet stem (hi MFMA only; both kernel forms) vs the fp32 conv 11x11/4
    + ReLU + max pool 3x3/2 of the same image; device-side window included."""
    from idunno.models.packed import pack_alex_stem_split

    torch.manual_seed(H + B + 2)
    img = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=DEV)
    w = torch.randn(64, 3, 11, 11) / (3 * 121) ** 0.5
    b = torch.randn(64) * 0.1
    fs, scale, bias, psum = pack_alex_stem_split(w.double(), b.double())
    fs, bias, psum = fs.to(DEV), bias.to(DEV), psum.to(DEV)
    ops.load().set_astem_f16_two_wg(two_wg)      # the kernel form (phased halves / two one-half workgroups)
    try:
        _alex_f16_case(ops, img, w, b, fs, scale, bias, psum, B)
    finally:
        ops.load().set_astem_f16_two_wg(True)


def _alex_f16_case(ops, img, w, b, fs, scale, bias, psum, B):
    from idunno.models.reference import preprocess_u8

    y = ops.alex_stem_u8_f16(img, fs, bias, psum, scale)
    x = preprocess_u8(img)
    ref = F.max_pool2d(F.relu(F.conv2d(x, w.to(DEV), b.to(DEV), 4, 2)), 3, 2, 0).permute(0, 2, 3, 1)
    assert y.dtype == torch.float16 and y.shape == ref.shape
    _check(y, ref)
    big = torch.cat([img.flip(0), img])
    st = torch.tensor([B + 3], dtype=torch.long, device=DEV)
    assert torch.equal(ops.alex_stem_u8_f16(big, fs, bias, psum, scale, st, B, 3), y)


def test_runner_fused_stem_matches_unfused(ops):
    from idunno.models import HipRunner, build_program

    p = build_program("resnet18", seed=11, randomize_bn=True)
    a, b = HipRunner(p, fuse_stem=True), HipRunner(p, fuse_stem=False)
    img = torch.randint(0, 256, (6, 224, 224, 3), dtype=torch.uint8, device=DEV)
    la, lb = a.logits(img), b.logits(img)
    assert (la - lb).abs().max().item() < 0.02 * lb.abs().max().item()
