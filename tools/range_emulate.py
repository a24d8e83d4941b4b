"""Per-rank cost of the key-range multi-GPU scheme, measured on ONE GPU.

The key-range scheme (genome_kmers.distributed.KeyRangeKmerSort) has no inter-GPU data path: rank
r's work is gk_shard_histogram over its position share plus gk_shard_sort_range over its digit
range.  Running every rank's share one after another on a single MI355X therefore measures each
rank's device time exactly; only the 2 KiB all-reduce is missing.  Prints one JSON line per N.

Usage: python tools/range_emulate.py [--genome-len L] [--worlds 1,2,4,8] [--reps 2]
"""

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "genome-kmers_amd"))
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=("c3", "c4", "c5"), default="c3")
    ap.add_argument("--genome-len", type=int, default=3_100_000_000)
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--worlds", type=str, default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()

    from genome_kmers import _native, synthetic
    from genome_kmers import distributed as D

    if args.config == "c3":
        sba, seg = synthetic.c3_genome(args.genome_len, 42)
    else:
        sba, seg = synthetic.grch38_surrogate(2)
    k = args.k or (63 if args.config == "c5" else 31)
    canonical = args.config == "c5"
    e = _native.Engine(0)
    e.set_sequence(sba, seg)
    e.sync()
    total = D.count_kmers(len(sba), seg, k)
    # single-GPU reference step for the same engine
    e.enumerate(k)
    e.sort(k, canonical=canonical)
    e.unique_count_only()
    e.sync()
    t0 = time.perf_counter()
    e.enumerate(k)
    e.sort(k, canonical=canonical)
    u1 = e.unique_count_only()
    e.sync()
    single_ms = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"single_gpu_ms": round(single_ms, 2), "kmers": total, "unique": u1}), flush=True)
    for world in [int(x) for x in args.worlds.split(",")]:
        pb = D.position_ranges(len(sba), world)
        per_rank = []
        uniq = 0
        kept = 0
        stages = None
        # the all-reduced histogram (every rank's share), outside the per-rank timings
        full = np.zeros(256, dtype=np.int64)
        for s in range(world):
            h, bits = e.shard_histogram(pb[s], pb[s + 1], k, canonical=canonical)
            full[:len(h)] += h.astype(np.int64)
        db = D.split_buckets(full[:1 << bits], world)
        for r in range(world):
            best = None
            for rep in range(args.reps + 1):  # the first one warms up
                e.sync()
                e.profile_enable(rep == args.reps)
                t0 = time.perf_counter()
                e.shard_histogram(pb[r], pb[r + 1], k, canonical=canonical)  # the rank's share of the all-reduce
                n = e.shard_sort_range(k, db[r], db[r + 1], canonical=canonical)
                u = e.unique_count_only()
                e.sync()
                dt = time.perf_counter() - t0
                if rep == args.reps:
                    rep_stages = e.profile_report()
                e.profile_enable(False)
                if rep > 0 and (best is None or dt < best):
                    best = dt
            if not per_rank or best * 1e3 > max(per_rank):
                stages = {name: round(v["total_ms"], 3) for name, v in rep_stages.items()}
            per_rank.append(round(best * 1e3, 2))
            uniq += u
            kept += n
        assert kept == total, (kept, total)  # every k-mer on exactly one rank
        worst = max(per_rank)
        print(json.dumps({"world": world, "per_rank_ms": per_rank, "max_rank_ms": worst,
                          "kmers_per_s": round(total / (worst * 1e-3), 1),
                          "speedup_vs_single": round(single_ms / worst, 2), "unique": uniq,
                          "slowest_rank_stages_ms": stages}), flush=True)


if __name__ == "__main__":
    main()
