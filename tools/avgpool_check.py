import torch, sys
sys.path.insert(0, '.')
from idunno import ops
ops.load()
for (B, HW, C) in [(400, 49, 512), (1024, 49, 2048), (7, 9, 96)]:
    x = torch.randn(B, HW, 1, C, device="cuda").half()
    y = ops.global_avgpool(x)
    ref = x.float().mean(dim=(1, 2))
    err = (y.float() - ref).abs().max().item()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3): ops.global_avgpool(x)
    st.record()
    for _ in range(50): ops.global_avgpool(x)
    en.record(); torch.cuda.synchronize()
    print(f"avgpool B={B} HW={HW} C={C}: err {err:.2e}  {st.elapsed_time(en)/50*1000:.1f} us", flush=True)
