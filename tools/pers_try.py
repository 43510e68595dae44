import sys, torch
sys.path.insert(0, ".")
from idunno import ops
from idunno.models.packed import pack_conv_weight
ext = ops.load()
print("experimental:", ext.has_experimental() if hasattr(ext, "has_experimental") else "?")
for (H, C, Co, res) in ((28, 512, 128, False), (14, 256, 1024, True), (56, 64, 256, True)):
    x = torch.randn(1024, H, H, C, device="cuda").half()
    w, _ = pack_conv_weight(torch.randn(Co, C, 1, 1) / C ** 0.5); w = w.cuda()
    b = torch.zeros(Co, device="cuda")
    r = torch.randn(1024, H, H, Co, device="cuda").half() if res else None
    ref = ops.conv2d(x, w, b, 1, 1, 1, 0, True, r, tile=36)
    for t in (70, 71, 72, 73):
        try:
            y = ops.conv2d(x, w, b, 1, 1, 1, 0, True, r, tile=t)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10): ops.conv2d(x, w, b, 1, 1, 1, 0, True, r, tile=t)
            e1.record(); torch.cuda.synchronize()
            print(H, C, Co, res, t, "ok", (y.float() - ref.float()).abs().max().item(), f"{e0.elapsed_time(e1)*100:.0f} us")
        except Exception as e:
            print(H, C, Co, res, t, "ERR", str(e)[:300])
