"""Probe: does torch's HIP init still work after many libgkm engines were created in the process?"""
import gc
import sys

import numpy as np

sys.path.insert(0, "genome-kmers_amd")
from genome_kmers import _native  # noqa: E402

keep = int(sys.argv[1]) if len(sys.argv) > 1 else 0
engines = []
for i in range(300):
    e = _native.Engine(0)
    e.set_sequence(np.frombuffer(b"ACGT" * 1000, dtype=np.uint8), np.zeros(1, dtype=np.uint32))
    e.enumerate(5)
    e.sort(5)
    if keep:
        engines.append(e)
    else:
        del e
    if i % 50 == 0:
        gc.collect()
        print("engines", i, flush=True)
import torch  # noqa: E402

print("torch device count", torch.cuda.device_count(), flush=True)
x = torch.zeros(4, device="cuda")
print("torch ok", x.sum().item(), flush=True)
