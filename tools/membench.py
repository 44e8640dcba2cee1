"""Write-bandwidth sanity check on the bench box: torch fill_ of the bench's output sizes."""
import torch

dev = torch.device("cuda:0")
for mb in (64, 256, 400, 1024):
    n = mb * 1024 * 1024 // 4
    t = torch.empty(n, device=dev)
    for _ in range(3):
        t.fill_(1.0)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        t.fill_(2.0)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    print(f"fill {mb} MB: {ms*1e3:.1f} us  {mb*1.048576/ms:.0f} GB/s", flush=True)
    del t
x = torch.empty(64, 512, 512, 3, device=dev)
y = torch.empty(64, 512, 512, device=dev)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    x.fill_(1.0)
    y.fill_(1.0)
e.record()
torch.cuda.synchronize()
print("rgb+depth fill", s.elapsed_time(e) / 10 * 1e3, "us")
