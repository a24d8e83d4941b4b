"""CPU baseline on prefixes of the C3 genome, outside the bench's budget.

The reference's sort (numba quicksort + compare_sba_kmers_lexicographically with validation,
kmers.py:1624-1731), as restated in oracle/gk_oracle.c (gcc -O3, 1 thread -- the reference is
single-threaded, kmers.py:1644-1648), timed on the first 1e8 and 3e8 bases of the C3 genome
(the reference's profiling genome, get_random_seq after np.random.seed(42):
genome_kmers.synthetic.c3_genome, the same stream as bench.py's C3; its prefixes are the genome's
first bases), and
extrapolated to the full 3,099,999,970 31-mers two ways, both labelled as extrapolations:
N log2 N from each prefix, and a power law fitted through the two prefixes (which carries the
growth of cache misses from 1e8 to 3e8 keys).

Usage (on the GPU box's host, ~10 min): python tools/cpu_baseline_prefixes.py [OUT.json]
"""

import json
import os
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "genome-kmers_amd"))
sys.path.insert(0, str(ROOT))

from genome_kmers import synthetic  # noqa: E402
from oracle import oracle  # noqa: E402

K = 31
N_FULL = 3_100_000_000 - K + 1


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def heartbeat(stop):
    """A progress line every 30 s while a long sort runs (ctypes releases the GIL)."""
    t0 = time.time()
    while not stop.wait(30):
        print(f"[cpu baseline] ... {time.time() - t0:.0f} s", file=sys.stderr, flush=True)


def main():
    out = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "profiles" / "r4" / "cpu_baseline_prefixes.json"
    runs = []
    for L in (100_000_000, 300_000_000):
        sba, _ = synthetic.c3_genome(L, 42)
        n = L - K + 1
        starts = np.arange(n, dtype=np.uint32)
        print(f"[cpu baseline] {L:,} bases, {n:,} k-mers: sorting ...", file=sys.stderr, flush=True)
        stop = threading.Event()
        hb = threading.Thread(target=heartbeat, args=(stop,), daemon=True)
        hb.start()
        t0 = time.perf_counter()
        got = oracle.quicksort(sba, starts, K, K)
        dt = time.perf_counter() - t0
        stop.set()
        hb.join()
        # spot check: windows of the sorted order are non-decreasing by bytes
        for off in (0, n // 2, n - 1000):
            w = got[off:off + 1000].astype(np.int64)
            rows = sba[w[:, None] + np.arange(K)[None, :]]
            assert all(bytes(rows[i]) <= bytes(rows[i + 1]) for i in range(len(rows) - 1))
        runs.append({"bases": L, "kmers": n, "seconds": round(dt, 2), "kmers_per_s": round(n / dt, 1)})
        print(f"[cpu baseline] {runs[-1]}", file=sys.stderr, flush=True)
        del sba, starts, got
    (n1, t1), (n2, t2) = [(r["kmers"], r["seconds"]) for r in runs]
    a = float(np.log(t2 / t1) / np.log(n2 / n1))
    nlogn = {f"from_{r['bases']:.0e}": round(r["seconds"] * (N_FULL * np.log2(N_FULL)) /
                                            (r["kmers"] * np.log2(r["kmers"])), 1) for r in runs}
    power = round(t2 * (N_FULL / n2) ** a, 1)
    res = {
        "what": "numba-quicksort restatement of Kmers.sort with validate_kmers (oracle/gk_oracle.c, gcc -O3), "
                "1 thread, on prefixes of the C3 genome, k = 31",
        "genome": "the reference's profiling genome: get_random_seq after np.random.seed(42) (MT19937)",
        "cpu_model": cpu_model(), "cores_on_box": os.cpu_count(), "threads_used": 1,
        "prefixes": runs,
        "full_workload": {
            "kmers": N_FULL,
            "seconds_nlog2n_extrapolated": nlogn,
            "seconds_power_law_extrapolated": power, "power_law_exponent": round(a, 3),
            "kmers_per_s_power_law": round(N_FULL / power, 1),
            "label": "extrapolated, not measured",
        },
    }
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
