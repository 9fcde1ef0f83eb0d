"""HBM write / read+write bandwidth probe (torch fill_ / copy_ on 2 GB buffers)."""
import torch
n = 1 << 29  # 2 GB fp32
a = torch.empty(n, device="cuda")
b = torch.empty(n, device="cuda")
for name, f, byts in (("write (fill_)", lambda: a.fill_(1.0), 4 * n), ("read+write (copy_)", lambda: b.copy_(a), 8 * n)):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"{name}: {byts / ms / 1e9:.2f} TB/s", flush=True)
