"""BN folding + MFMA weight packing, checked on CPU by re-running the packed
program with fp32 torch ops (idunno.models.packed.emulate)."""
import pytest
import torch

from idunno.models import packed
from idunno.models import reference as ref


@pytest.mark.parametrize("name", ["resnet18", "alexnet", "resnet50"])
def test_packed_program_matches_reference(name):
    m = ref.build(name, seed=1, randomize_bn=True)
    p = packed.compile_model(m, name)
    torch.manual_seed(0)
    img = torch.randint(0, 256, (2, 224, 224, 3), dtype=torch.uint8)
    with torch.no_grad():
        r = m(ref.preprocess_u8(img))
    e = packed.emulate(p, img)
    assert (r - e).abs().max().item() < 2e-3 * r.abs().max().item()
    assert torch.equal(r.argmax(1), e.argmax(1))


def test_pack_unpack_roundtrip_small_and_big():
    for shape in [(64, 3, 7, 7), (64, 3, 11, 11), (128, 64, 3, 3), (256, 128, 1, 1)]:
        w = torch.randn(*shape)
        pw, small = packed.pack_conv_weight(w)
        c = packed.Conv(pw, torch.zeros(shape[0]), shape[1], shape[0], shape[2], shape[3], 1, 0, False, small)
        assert small == (shape[1] == 3)
        assert torch.equal(packed.unpack_conv_weight(c), w.half().float())
    assert packed.pack_conv_weight(torch.randn(64, 3, 7, 7))[0].shape == (64, 7 * 32)
    assert packed.pack_conv_weight(torch.randn(64, 3, 11, 11))[0].shape == (64, 11 * 64)


def test_flops():
    p = packed.build_program("resnet18")
    assert abs(packed.program_flops(p) / 1e9 - 3.63) < 0.02
    p = packed.build_program("alexnet")
    assert abs(packed.program_flops(p) / 1e9 - 1.43) < 0.02


def test_alias():
    assert ref.canonical("resnet") == "resnet18"
    with pytest.raises(ValueError):
        ref.canonical("vgg")


def test_concurrent_builds_give_identical_weights():
    """Nodes of one process build their models on their own threads; the
    global-RNG init must not interleave (was: wrong answers in LocalCluster)."""
    import threading

    from idunno.models import reference as ref

    out = [None] * 4

    def work(i):
        out[i] = ref.build("resnet18", seed=0).state_dict()

    ths = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for sd in out[1:]:
        assert all(torch.equal(sd[k], out[0][k]) for k in out[0])


@pytest.mark.parametrize("name", ["resnet18", "alexnet"])
def test_fp32_program_is_exact_fold_of_reference(name):
    """dtype "fp32": weights stay fp32 (no rounding), so the emulated packed
    program matches the module to fp32 folding error only."""
    m = ref.build(name, seed=2, randomize_bn=True)
    p = packed.compile_model(m, name, dtype="fp32")
    assert p.dtype == "fp32"
    assert all(c.w.dtype == torch.float32 for c in p.all_convs())
    torch.manual_seed(1)
    img = torch.randint(0, 256, (2, 224, 224, 3), dtype=torch.uint8)
    with torch.no_grad():
        r = m(ref.preprocess_u8(img))
    e = packed.emulate(p, img)
    assert (r - e).abs().max().item() < 1e-4 * r.abs().max().item()


def test_pack_unpack_roundtrip_fp32():
    for shape in [(64, 3, 7, 7), (64, 3, 11, 11), (12, 3, 5, 5), (128, 64, 3, 3), (20, 48, 3, 3)]:
        w = torch.randn(*shape)
        pw, small = packed.pack_conv_weight(w, "fp32")
        assert pw.dtype == torch.float32
        c = packed.Conv(pw, torch.zeros(shape[0]), shape[1], shape[0], shape[2], shape[3], 1, 0, False, small)
        assert small == (shape[1] == 3)
        assert torch.equal(packed.unpack_conv_weight(c), w)
    # small-C rows are 4 taps x 4 channels: kw 7 -> 8 taps, 11 -> 12 taps
    assert packed.pack_conv_weight(torch.randn(64, 3, 7, 7), "fp32")[0].shape == (64, 7 * 2 * 16)
    assert packed.pack_conv_weight(torch.randn(64, 3, 11, 11), "fp32")[0].shape == (64, 11 * 3 * 16)
    with pytest.raises(ValueError):
        packed.pack_conv_weight(torch.randn(8, 20, 3, 3), "fp32")
    with pytest.raises(ValueError):
        packed.pack_conv_weight(torch.randn(8, 64, 3, 3), "bf8")


def _pack3_geometry(W, KW, stride, pad, E=4):
    g = 1
    while g < E and (3 * stride) % (2 * g) == 0:
        g *= 2
    return E // g, (3 * (W + 2 * pad) + 2 * E - 2) // E * E, (3 * KW + E - 1) // E, g


def _emulate_pack3(img, w, b, stride, pad, dtype="fp32"):
    """The packed-row stem (preprocess_pack3 + conv_f32 mode 2 / conv_glds
    pack3) index math in torch: row copies, aligned chunk starts, (kh, chunk)
    K order."""
    E = 4 if dtype == "fp32" else 8
    B, H, W, _ = img.shape
    cout, _, KH, KW = w.shape
    nc, wp, cpk, g = _pack3_geometry(W, KW, stride, pad, E)
    x = ref.preprocess_u8(img).permute(0, 2, 3, 1).reshape(B, H, 3 * W)
    R = torch.zeros(B, H, 3 * (W + 2 * pad) + 4 * E)
    R[:, :, 3 * pad:3 * pad + 3 * W] = x
    x3 = torch.stack([R[:, :, c * g:c * g + wp] for c in range(nc)], 2)       # [B, H, nc, wp]
    assert x3.shape == (B, H, nc, wp)
    wpk = packed.pack_conv_weight_p3(w, dtype).float()
    stage = 16 if dtype == "fp32" else 64
    nk = (KH * cpk * E + stage - 1) // stage
    assert wpk.shape == (cout, nk * stage)
    Ho, Wo = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1
    out = torch.zeros(B, Ho, Wo, cout)
    for oh in range(Ho):
        for ow in range(Wo):
            r0 = 3 * stride * ow
            sh = r0 % E
            assert (r0 - sh) % E == 0 and sh % g == 0
            vec = torch.zeros(B, nk * stage)
            for kh in range(KH):
                ih = oh * stride - pad + kh
                if 0 <= ih < H:
                    vec[:, kh * E * cpk:(kh + 1) * E * cpk] = x3[:, ih, sh // g, r0 - sh:r0 - sh + E * cpk]
            out[:, oh, ow] = vec @ wpk.t() + b
    return out


@pytest.mark.parametrize("dtype", ["fp32", "fp16"])
@pytest.mark.parametrize("H,W,KH,KW,stride,pad", [(23, 21, 7, 7, 2, 3), (31, 27, 11, 11, 4, 2), (9, 12, 5, 5, 1, 2)])
def test_pack3_stem_layout_matches_conv(H, W, KH, KW, stride, pad, dtype):
    if dtype == "fp16" and not packed.pack3_eligible(3, KW, stride, dtype):
        pytest.skip("fp16 packed rows need an even stride")
    torch.manual_seed(H + W)
    img = torch.randint(0, 256, (2, H, W, 3), dtype=torch.uint8)
    w = torch.randn(8, 3, KH, KW)
    b = torch.randn(8)
    ref_out = torch.nn.functional.conv2d(ref.preprocess_u8(img), w, b, stride, pad).permute(0, 2, 3, 1)
    e = _emulate_pack3(img, w, b, stride, pad, dtype)
    tol = 1e-4 if dtype == "fp32" else 2e-3          # fp16: rounded weights
    assert (e - ref_out).abs().max().item() < tol * ref_out.abs().max().item()
