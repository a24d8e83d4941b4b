"""Probe (tuning): random 32-B row gathers from a large table with torch (index_select), against
the byte-window gather of the key re-encode.  Prints GB/s and rows/s."""
import time
import torch

n = 1_000_000_000
dev = torch.device("cuda", 0)
tab = torch.empty((n, 4), dtype=torch.int64, device=dev)
tab.random_()
idx = torch.randint(0, n, (n,), device=dev, dtype=torch.int64)
out = torch.empty((n, 4), dtype=torch.int64, device=dev)
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.index_select(tab, 0, idx, out=out)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"index_select 32-B rows: {dt*1e3:.1f} ms, {n/dt/1e9:.2f} G rows/s, {n*32/dt/1e12:.2f} TB/s useful", flush=True)
# sequential for comparison
torch.cuda.synchronize()
t0 = time.perf_counter()
out.copy_(tab)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"copy: {dt*1e3:.1f} ms, {2*n*32/dt/1e12:.2f} TB/s", flush=True)
