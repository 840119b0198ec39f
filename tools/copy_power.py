"""Reference power point for tools/power_probe.sh: torch's device copy of the C2 arena (256 MiB in,
256 MiB out) back to back, as a linear streaming access pattern at HBM rate."""
import sys
import time

import torch

n = 256 << 20
a = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
b = torch.empty_like(a)
c = torch.empty_like(a)
for _ in range(50):
    b.copy_(a)
torch.cuda.synchronize()
secs = float(sys.argv[1]) if len(sys.argv) > 1 else 14.0
t0 = time.perf_counter()
k = 0
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
while time.perf_counter() - t0 < secs:
    for _ in range(200):
        (b if k % 2 == 0 else c).copy_(a if k % 2 == 0 else b)
        k += 1
    torch.cuda.synchronize()
e1.record()
e1.synchronize()
us = e0.elapsed_time(e1) * 1e3 / k
print({"copy_us": round(us, 2), "GBs": round(2 * n / us / 1e3, 1)})
