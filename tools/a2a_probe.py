"""Probe: world-1 RCCL all_to_all_single correctness at large message sizes (development tool)."""
import os
import sys

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
for n in [int(x) for x in sys.argv[1:]]:
    src = torch.arange(n, dtype=torch.int64, device="cuda")
    dst = torch.zeros_like(src)
    dist.all_to_all_single(dst, src, [n], [n])
    torch.cuda.synchronize()
    bad = int((dst != src).sum().item())
    print(f"n={n:,} int64 bytes={8 * n:,} mismatches={bad:,}", flush=True)
    del src, dst
dist.destroy_process_group()
