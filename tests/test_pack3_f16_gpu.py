"""fp16 RGB stems on packed rows (preprocess_pack3 f16 + conv_glds pack3) vs
the fp64 oracle of the same fp16-rounded operands."""
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


@pytest.mark.parametrize("tile", [-1, 23, 27, 31, 33, 35])
@pytest.mark.parametrize("B,H,W,k,s,p,Cout", [
    (2, 224, 224, 11, 4, 2, 64),    # AlexNet conv1
    (2, 224, 224, 7, 2, 3, 64),     # ResNet stem shape (4 row copies)
    (1, 37, 29, 7, 2, 3, 64),       # ragged image, padding on every border
])
def test_conv_f16_pack3(ops, tile, B, H, W, k, s, p, Cout):
    from idunno.models.packed import pack_conv_weight_p3
    from idunno.models.reference import preprocess_u8

    torch.manual_seed(H + k + tile)
    img = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=DEV)
    w = torch.randn(Cout, 3, k, k) / (3 * k * k) ** 0.5
    b = torch.randn(Cout) * 0.1
    x3 = ops.preprocess_pack3(img, k, s, p, f16=True)
    assert x3.dtype == torch.float16
    y = ops.conv2d_pack3(x3, pack_conv_weight_p3(w, "fp16").to(DEV), b.to(DEV), W, k, k, s, p, True, tile)
    xin = preprocess_u8(img).half().double()                    # the operands the kernel sees
    ref = F.relu(F.conv2d(xin, w.half().double().to(DEV), b.double().to(DEV), s, p)).permute(0, 2, 3, 1)
    assert y.shape == ref.shape and y.dtype == torch.float16
    err = (y.double() - ref).abs().max().item()
    assert err <= 2e-3 * ref.abs().max().item() + 2e-3, err


def test_preprocess_pack3_f16_window(ops):
    torch.manual_seed(12)
    shard = torch.randint(0, 256, (10, 30, 34, 3), dtype=torch.uint8, device=DEV)
    start = torch.tensor([203], dtype=torch.int64, device=DEV)
    a = ops.preprocess_pack3(shard, 11, 4, 2, start, 4, 200, f16=True)
    b = ops.preprocess_pack3(shard[3:7].contiguous(), 11, 4, 2, f16=True)
    assert torch.equal(a, b)
    f = ops.preprocess_pack3(shard[3:7].contiguous(), 11, 4, 2)          # fp32 copy of the same rows
    assert f.shape[:2] == b.shape[:2]


def test_runner_alexnet_f16_pack3_vs_nhwc4(ops):
    from idunno.models import HipRunner, build_program

    p = build_program("alexnet", seed=4, randomize_bn=True, dtype="fp16")
    img = ops.synth_images(8, 0, 6, DEV)
    ra = HipRunner(p)
    ra.pack3_f16 = True
    a = ra.logits(img).float()
    b = HipRunner(p).logits(img).float()
    assert (a - b).abs().max().item() <= 1e-2 * b.abs().max().item()
