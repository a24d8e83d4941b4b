"""One key-range rank's device work, repeated (profiling target for rocprofv3; tuning only).

Usage: python tools/range_rank.py [--config c3|c4] [--world 8] [--rank 0] [--reps 3]
"""

import argparse
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "genome-kmers_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=("c3", "c4"), default="c3")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from genome_kmers import _native, synthetic
    from genome_kmers import distributed as D

    sba, seg = synthetic.c3_genome(3_100_000_000, 42) if args.config == "c3" else synthetic.grch38_surrogate(2)
    k, w, r = 31, args.world, args.rank
    e = _native.Engine(0)
    e.set_sequence(sba, seg)
    e.sync()
    pb = D.position_ranges(len(sba), w)
    mixed = not e.is_acgt()
    full = np.zeros(4096, dtype=np.int64)
    rests, runs_l = [], []
    for s in range(w):
        h, bits = e.shard_histogram(pb[s], pb[s + 1], k)
        h = np.asarray(h, dtype=np.uint64)
        if mixed:
            rest, runs = e.shard_class_b(pb[s], pb[s + 1], k, h)
            rests.append(rest)
            runs_l.append(runs)
        full[:len(h)] += h.astype(np.int64)
    db = D.split_buckets(full[:1 << bits], w)
    for i in range(args.reps):
        e.sync()
        t0 = time.perf_counter()
        e.shard_histogram(pb[r], pb[r + 1], k)
        if mixed:
            n = e.shard_sort_range_b(k, db[r], db[r + 1], np.concatenate(rests), np.concatenate(runs_l), False)
        else:
            n = e.shard_sort_range(k, db[r], db[r + 1])
        e.materialize_keys()
        u = e.unique_count_only()
        e.sync()
        print(f"rep {i}: rank {r}/{w} kept {n} unique {u} in {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
