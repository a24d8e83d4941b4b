"""Where the end-to-end interval of a C3 sort goes (sort hint on / off): wall time of gk_set_sequence,
of the device catching up after it (a sync), and of the step, with the profile's stage times.
Tuning only.  Usage: python tools/e2e_probe.py [--regions 16,32] [--reps 3] [--genome-len N] [--pageable]
(--pageable: the source is the caller's pageable numpy array instead of pinned memory)"""

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "genome-kmers_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--regions", default="16")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--genome-len", type=int, default=3_100_000_000)
    ap.add_argument("--k", type=int, default=31)
    ap.add_argument("--pageable", action="store_true")
    a = ap.parse_args()
    import torch
    from genome_kmers import _native, synthetic

    sba, seg = synthetic.c3_genome(a.genome_len, 42)
    pinned = torch.empty(len(sba), dtype=torch.uint8).pin_memory()
    pinned.numpy()[:] = sba
    src = sba if a.pageable else pinned.numpy()
    eng = _native.Engine(0)
    k = a.k

    def step():
        eng.enumerate(k)
        eng.sort(k)
        eng.materialize_keys()
        eng.unique_count_only()

    eng.set_sequence(src, seg)
    step()
    eng.sync()
    for regions in [0] + [int(x) for x in a.regions.split(",")]:
        os.environ["GKM_PREFETCH_REGIONS"] = str(max(regions, 1))
        eng.sort_hint(k if regions else 0)
        for rep in range(a.reps):
            eng.profile_enable(True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.set_sequence(src, seg)
            t1 = time.perf_counter()
            eng.sync()
            t2 = time.perf_counter()
            step()
            eng.sync()
            t3 = time.perf_counter()
            r = eng.profile_report()
            eng.profile_enable(False)
            st = {n: round(v["total_ms"], 2) for n, v in sorted(r.items()) if v["total_ms"] > 0.3}
            print(json.dumps({"source": "pageable" if a.pageable else "pinned", "regions": regions, "set_sequence_ms": round((t1 - t0) * 1e3, 2),
                              "catch_up_ms": round((t2 - t1) * 1e3, 2), "step_ms": round((t3 - t2) * 1e3, 2),
                              "e2e_with_sync_ms": round((t3 - t0) * 1e3, 2), "stages": st}), flush=True)
    eng.sort_hint(0)


if __name__ == "__main__":
    main()
