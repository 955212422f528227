"""Does data stay in the XCD L2s across kernel launches?  Repeated torch reductions over buffers of
1/4/8/16/64/1024 MB; per-launch time and effective bandwidth from HIP events."""
import torch

dev = torch.device("cuda:0")
for mb in [1, 4, 8, 16, 24, 32, 64, 128, 1024]:
    x = torch.rand(mb * 262144, device=dev)
    out = torch.empty((), device=dev)
    for _ in range(5):
        torch.sum(x, 0, out=out)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    s.record()
    for _ in range(n):
        torch.sum(x, 0, out=out)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1000 / n
    print(f"{mb:5d} MB  {us:8.1f} us/launch  {mb * 1.048576e6 / (us * 1e-6) / 1e12:6.2f} TB/s", flush=True)
