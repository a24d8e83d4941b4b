"""gk_set_sequence's packed transfer of the 3.1 Gb C3 genome at several host thread counts
(GKM_XFER_THREADS), from pageable numpy memory (packed chunks only) and from pinned memory (packed
chunks from the front, raw DMA from the back); best of 3 each, device synchronised."""

import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "genome-kmers_amd"))

from genome_kmers import _native, synthetic  # noqa: E402

import torch  # noqa: E402

sba, seg = synthetic.c3_genome()
pinned = torch.empty(len(sba), dtype=torch.uint8).pin_memory()
pinned.numpy()[:] = sba
eng = _native.Engine()
out = {}
numa = os.environ.get("XFER_NUMA_AB") == "1"  # also each count with GKM_XFER_NUMA=1
for src_name, src in (("pageable", sba), ("pinned", pinned.numpy())):
    for t in [f"{a}{b}" for a in (sys.argv[1:] or ["1", "4", "8", "16", "32"]) for b in (("", "n") if numa else ("",))]:
        os.environ["GKM_XFER_NUMA"] = "1" if t.endswith("n") else "0"
        os.environ["GKM_XFER_THREADS"] = t.rstrip("n")
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            eng.set_sequence(src, seg)
            eng.sync()
            best = min(best, time.perf_counter() - t0)
        out[f"{src_name}_{t}"] = round(best * 1e3, 1)
        print(f"{src_name} threads {t}: {best * 1e3:.1f} ms ({len(sba) / best / 1e9:.1f} GB/s)", flush=True)
print(json.dumps({"set_sequence_ms": out, "cpus": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}))
