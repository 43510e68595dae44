#!/usr/bin/env python3
"""CPU emulation of a split-fp16 Winograd F(2x2,3x3) conv (VERDICT r3 item 1,
lever (a)): fp32 input transform, V and U split to (hi, lo) halfs, the
e-GEMMs as hi*hi + hi*lo + lo*hi with fp32 accumulation, fp32 output
transform -- against the split direct conv and torch fp32, all vs fp64, per
ResNet18 3x3/s1 layer shape.  Prints max |err| / max |ref| per layer.
Result (round 4): the Winograd form doubles the per-layer error of the split
direct conv (3.4-5.2e-7 vs 1.8-3.1e-7; torch fp32 1.7-2.5e-7), see
docs/KERNELS.md "Split Winograd: numerics and budget".

usage: python tools/wino_split_numerics.py
"""
import torch, math
torch.manual_seed(0)
def f16split(x):
    hi = x.to(torch.float16).to(torch.float64)
    lo = (x - hi).to(torch.float16).to(torch.float64)
    return hi, lo
def conv_direct_split(x, w):
    # x: [B,C,H,W] fp64 (values representable as split), w [N,C,3,3]
    s = 2.0 ** (13 - math.ceil(math.log2(w.abs().max().item())))
    wh, wl = f16split(w * s)
    xh, xl = f16split(x)
    f = lambda a, b: torch.nn.functional.conv2d(a.float(), b.float(), padding=1).double()
    # fp32 accumulate (approx): each product exact in fp32, sum rounding fp32
    return (f(xh, wh) + f(xh, wl) + f(xl, wh)) / s
def conv_wino_split(x, w, vsplit=True, f32_input=True):
    B, C, H, W = x.shape
    N = w.shape[0]
    G = torch.tensor([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], dtype=torch.float64)
    Bt = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float64)
    At = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float64)
    U = torch.einsum('ei,ncij,fj->efnc', G, w, G)  # [4,4,N,C]
    s = 2.0 ** (13 - math.ceil(math.log2(U.abs().max().item())))
    Uh, Ul = f16split(U * s)
    xp = torch.nn.functional.pad(x, (1, 1 + (W % 2), 1, 1 + (H % 2)))
    TY, TX = (H + 1) // 2, (W + 1) // 2
    # patches d: [B,C,TY,TX,4,4]
    d = xp.unfold(2, 4, 2).unfold(3, 4, 2)
    if not f32_input:
        dh, dl = f16split(d); d = dh + dl
    d = d.float()
    t = torch.einsum('ei,bcyxij->bcyxej', Bt.float(), d)   # fp32 (sum of 2 terms: one rounding)
    V = torch.einsum('bcyxej,fj->bcyxef', t, Bt.float()).double()
    if vsplit:
        Vh, Vl = f16split(V)
    else:
        Vh, Vl = V, torch.zeros_like(V)
    mm = lambda u, v: torch.einsum('efnc,bcyxef->bnyxef', u.float(), v.float()).double()
    M = (mm(Uh, Vh) + mm(Uh, Vl) + mm(Ul, Vh)).float()
    Y = torch.einsum('pe,bnyxef,qf->bnyxpq', At.float(), M, At.float()).double() / s
    Y = Y.permute(0, 1, 2, 4, 3, 5).reshape(B, N, 2 * TY, 2 * TX)[:, :, :H, :W]
    return Y
for (C, H) in [(64, 56), (128, 28), (256, 14), (512, 7)]:
    B = 2
    x = torch.relu(torch.randn(B, C, H, H, dtype=torch.float64))
    xh, xl = f16split(x); x = xh + xl  # activations are stored split
    w = torch.randn(C, C, 3, 3, dtype=torch.float64) * math.sqrt(2.0 / (9 * C))
    ref = torch.nn.functional.conv2d(x, w, padding=1)
    scale = ref.abs().max().item()
    e_dir = (conv_direct_split(x, w) - ref).abs().max().item() / scale
    e_w = (conv_wino_split(x, w) - ref).abs().max().item() / scale
    e_w32 = (torch.nn.functional.conv2d(x.float(), w.float(), padding=1).double() - ref).abs().max().item() / scale
    print(f"C={C} H={H}: direct split {e_dir:.2e}  wino split {e_w:.2e}  torch fp32 {e_w32:.2e}")
