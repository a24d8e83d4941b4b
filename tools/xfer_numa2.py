"""Where the source pages of gk_set_sequence live, and the packed transfer with the packing threads
unplaced (GKM_XFER_NUMA=0), on the caller's node (1) and on the source buffer's node (2), from the
caller's pageable numpy sba, torch pinned memory and hipHostRegister'ed numpy memory; 3.1 Gb C3
genome, best of 3 each, device synchronised."""

import ctypes
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "genome-kmers_amd"))

from genome_kmers import _native, synthetic  # noqa: E402

import torch  # noqa: E402

libc = ctypes.CDLL(None, use_errno=True)
SYS_get_mempolicy = 239  # x86_64


def nodes(arr: np.ndarray, samples: int = 33) -> dict:
    base = arr.ctypes.data
    out = {}
    for i in range(samples):
        addr = base + (arr.nbytes - 1) * i // (samples - 1)
        node = ctypes.c_int(-1)
        r = libc.syscall(SYS_get_mempolicy, ctypes.byref(node), None, ctypes.c_ulong(0), ctypes.c_void_p(addr),
                         ctypes.c_ulong(3))
        key = int(node.value) if r == 0 else "err"
        out[key] = out.get(key, 0) + 1
    return out


sba, seg = synthetic.c3_genome()
pinned = torch.empty(len(sba), dtype=torch.uint8).pin_memory()
pinned.numpy()[:] = sba
reg = np.empty_like(sba)
reg[:] = sba
cudart = torch.cuda.cudart()
rc = cudart.cudaHostRegister(reg.ctypes.data, reg.nbytes, 0)
print(f"hostRegister rc {rc}", flush=True)
print("caller cpu", os.sched_getcpu() if hasattr(os, "sched_getcpu") else "?", flush=True)
srcs = (("pageable", sba), ("pinned", pinned.numpy()), ("registered", reg))
for name, src in srcs:
    print(f"{name}: page nodes {nodes(src)}", flush=True)
eng = _native.Engine()
out = {}
for name, src in srcs:
    for mode in ("0", "1", "2"):
        os.environ["GKM_XFER_NUMA"] = mode
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            eng.set_sequence(src, seg)
            eng.sync()
            best = min(best, time.perf_counter() - t0)
        out[f"{name}_numa{mode}"] = round(best * 1e3, 1)
        print(f"{name} GKM_XFER_NUMA={mode}: {best * 1e3:.1f} ms ({len(sba) / best / 1e9:.1f} GB/s)", flush=True)
print(json.dumps({"set_sequence_ms": out}))
