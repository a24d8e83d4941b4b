"""Time gk_sort(k, GK_SORT_QUICKSORT_ORDER) -- the reference's own (numba quicksort) tie order -- on
a prefix of the C3 genome, beside the default stable sort of the same k-mers, and check that the two
differ only inside groups of equal k-mers (same k-mer sequence).  Usage:
python tools/qorder_time.py [L] [k]   (default 1e8 bases, k = 31)"""

import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "genome-kmers_amd"))


def main():
    from genome_kmers import _native, synthetic

    L = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 31
    sba, seg = synthetic.c3_genome(L, 42)
    eng = _native.Engine(0)
    eng.set_sequence(sba, seg)
    out = {"bases": L, "k": k}
    res = {}
    for name, qs in (("stable", False), ("reference_quicksort_order", True)):
        n = eng.enumerate(k)
        eng.sync()
        t0 = time.perf_counter()
        eng.sort(k, quicksort_order=qs)
        eng.sync()
        out[f"{name}_s"] = round(time.perf_counter() - t0, 3)
        res[name] = eng.copy_starts(np.empty(n, dtype=np.uint32))
    a, b = res["stable"], res["reference_quicksort_order"]
    out["kmers"] = int(len(a))
    out["same_multiset"] = bool(np.array_equal(np.sort(a), np.sort(b)))
    diff = np.flatnonzero(a != b)
    out["positions_differing"] = int(len(diff))
    if len(diff):  # every differing position holds the same k-mer in both orders
        sel = diff[:: max(1, len(diff) // 20000)]
        rows_a = sba[a[sel].astype(np.int64)[:, None] + np.arange(k)]
        rows_b = sba[b[sel].astype(np.int64)[:, None] + np.arange(k)]
        out["differences_inside_tie_groups"] = bool(np.array_equal(rows_a, rows_b))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
