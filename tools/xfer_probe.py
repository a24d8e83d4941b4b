"""gk_set_sequence of the 3.1 Gb C3 genome from pinned host memory: median of 7 transfers per host
packer implementation (GKM_PACK_IMPL, read once per process: one child process each) and thread
count (GKM_XFER_THREADS).  Tuning only.  Usage: python tools/xfer_probe.py [impl:threads ...]"""
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def child():
    sys.path.insert(0, str(ROOT / "genome-kmers_amd"))
    import numpy as np
    import torch
    from genome_kmers import _native, synthetic

    sba, seg = synthetic.c3_genome(3_100_000_000, 42)
    pinned = torch.empty(len(sba), dtype=torch.uint8).pin_memory()
    pinned.numpy()[:] = sba
    eng = _native.Engine(0)
    ts = []
    for _ in range(8):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.set_sequence(pinned.numpy(), seg)
        eng.sync()
        ts.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"impl": os.environ.get("GKM_PACK_IMPL", "default"),
                      "threads": os.environ.get("GKM_XFER_THREADS", "16"),
                      "median_ms": round(float(np.median(ts[1:])), 2), "all_ms": [round(x, 2) for x in ts]}))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
    else:
        for spec in sys.argv[1:] or ["avx2:16", "avx512:16"]:
            impl, thr = spec.split(":")
            env = dict(os.environ, GKM_PACK_IMPL=impl, GKM_XFER_THREADS=thr)
            r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True)
            print(r.stdout.strip() or r.stderr[-500:], flush=True)
