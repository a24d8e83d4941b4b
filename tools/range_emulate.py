"""Per-rank cost of the multi-GPU schemes, measured on ONE GPU.

Every rank's device work runs on a single MI355X one after another, so each rank's device time is
measured exactly; what a real N-GPU run adds is the collective:

  --scheme range (KeyRangeKmerSort): gk_shard_histogram over the rank's position share (on a mixed
      sba also gk_shard_class_b: the share's class-B lists), then gk_shard_sort_range (mixed:
      gk_shard_sort_range_b with every share's lists) over its digit range (keys materialised,
      unique counts); the collectives -- the 32 KiB all-reduce of the histograms, on a mixed sba
      the all-gathers of the list sizes and lists, and the closing barrier -- are added as
      collective_ms: a MEASURED one-rank RCCL run of the same calls (launch + host round trips) plus
      a MODELLED ring cost per extra rank (RING_STEP_US per step, bytes at one xGMI link).
  --scheme a2a (ShardedKmerSort): gk_shard_partition of the rank's position share, then
      gk_shard_sort of the buckets it owns (pieces sliced from every rank's send buffer on the same
      GPU); the missing collective is the all-to-all, reported as a link-bound estimate: the
      largest per-peer message of the rank (send or receive) / 153 GB/s (one xGMI link per peer,
      MI355X_MICROARCH.md), which no RCCL run can beat.

The single-GPU step (enumerate + sort + keys + unique counts, as bench.py) and every rank are timed
as the best of --reps runs after one warm-up.  Prints one JSON line per N.

Usage: python tools/range_emulate.py [--config c3|c4|c5] [--scheme range|a2a] [--worlds 8,4,2] [--reps 2]
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

LINK_GBS = 153.0  # one xGMI link, per direction (MI355X_MICROARCH.md)
RING_STEP_US = 10.0  # assumed latency of one ring step of a small RCCL collective over xGMI (modelled)


def measure_collectives(reps=20):
    """One-rank RCCL (world size 1) all-reduce of the 4096-bin histogram, two all-gathers and a
    barrier, as KeyRangeKmerSort.run issues them: the launch and host round-trip part of the
    collectives, measured (ms, best of reps)."""
    import socket

    import torch
    import torch.distributed as dist

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    dev = torch.device("cuda", 0)
    h = torch.zeros(4096, dtype=torch.int64, device=dev)
    sz = torch.zeros(2, dtype=torch.int64, device=dev)
    lst = torch.zeros(1024, dtype=torch.int32, device=dev)
    out = {}
    for name, fn in (("all_reduce", lambda: (dist.all_reduce(h), h.cpu())),
                     ("all_gather_pair", lambda: (dist.all_gather([torch.empty_like(sz)], sz), sz.cpu(),
                                                  dist.all_gather([torch.empty_like(lst)], lst), lst.cpu())),
                     ("barrier", lambda: dist.barrier())):
        best = None
        for _ in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            best = dt if best is None else min(best, dt)
        out[name] = round(best, 4)
    dist.destroy_process_group()
    return out


def collective_ms(world, measured, gather_bytes, mixed):
    """Measured one-rank cost + modelled ring steps: all-reduce 2 (N - 1) steps, all-gather N - 1
    each, barrier ~ an all-reduce of nothing; bytes at one xGMI link."""
    steps = 2 * (world - 1) + (2 * (world - 1) if mixed else 0) + 2 * (world - 1)
    wire = (2 * (world - 1) / world * 32768 + ((world - 1) / world * gather_bytes if mixed else 0)) / (LINK_GBS * 1e9)
    base = measured["all_reduce"] + measured["barrier"] + (measured["all_gather_pair"] if mixed else 0)
    return base + steps * RING_STEP_US * 1e-3 + wire * 1e3


def best_of(fn, reps, sync):
    best, out = None, None
    for rep in range(reps + 1):  # the first one warms up
        sync()
        t0 = time.perf_counter()
        out = fn(rep == reps)
        sync()
        dt = time.perf_counter() - t0
        if rep > 0 and (best is None or dt < best):
            best = dt
    return best * 1e3, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=("c3", "c4", "c5"), default="c3")
    ap.add_argument("--scheme", choices=("range", "a2a"), default="range")
    ap.add_argument("--genome-len", type=int, default=3_100_000_000)
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--worlds", type=str, default="8,4,2")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--keys", action="store_true",
                    help="a2a: exchange (key, start) pairs (12 B) even where the starts alone (4 B, "
                         "GK_SHARD_STARTS_ONLY, the default for forward ACGT k <= 32) would do")
    ap.add_argument("--b-scan", action="store_true",
                    help="mixed sba: every rank scans the whole sequence for its class-B k-mers (round-2 path)")
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

    def single(_last):
        e.enumerate(k)
        e.sort(k, canonical=canonical)
        e.materialize_keys()
        return e.unique_count_only()

    single_ms, u1 = best_of(single, args.reps, e.sync)
    mixed = not e.is_acgt() and k >= 4 and not args.b_scan
    measured = measure_collectives() if args.scheme == "range" else None
    print(json.dumps({"config": args.config, "scheme": args.scheme, "single_gpu_ms": round(single_ms, 2),
                      "kmers": total, "unique": u1, "timing": f"best of {args.reps} after a warm-up",
                      "collectives_one_rank_ms": measured, "ring_step_us_modelled": RING_STEP_US,
                      "label": "per-rank emulation on one GPU; unmeasured on multi-GPU hardware"}), flush=True)

    for world in [int(x) for x in args.worlds.split(",")]:
        pb = D.position_ranges(len(sba), world)
        per_rank, extra, stages, uniq, kept = [], [], None, 0, 0

        all_stages = []

        def record(ms, rep_stages):
            nonlocal stages
            st = {name: round(v["total_ms"], 3) for name, v in rep_stages.items()}
            if not per_rank or ms > max(per_rank):
                stages = st
            all_stages.append(st)
            per_rank.append(round(ms, 2))

        if args.scheme == "range":
            full = np.zeros(4096, dtype=np.int64)
            rests, runs_l = [], []
            for s in range(world):
                h, bits = e.shard_histogram(pb[s], pb[s + 1], k, canonical=canonical)
                h = np.asarray(h, dtype=np.uint64)
                if mixed:
                    rest, runs = e.shard_class_b(pb[s], pb[s + 1], k, h, canonical=canonical)
                    rests.append(rest)
                    runs_l.append(runs)
                full[:len(h)] += h.astype(np.int64)
            db = D.split_buckets(full[:1 << bits], world)
            rest_all = np.concatenate(rests) if mixed else None
            runs_all = np.concatenate(runs_l).reshape(-1, 3) if mixed else None
            gather_bytes = (4 * len(rest_all) + 12 * len(runs_all)) if mixed else 0
            coll = collective_ms(world, measured, gather_bytes, mixed)
            for r in range(world):
                print(f"# world {world}: rank {r}", file=sys.stderr, flush=True)  # progress (long runs)

                def rank(last, r=r):
                    e.profile_enable(last)
                    h, _ = e.shard_histogram(pb[r], pb[r + 1], k, canonical=canonical)  # the rank's share
                    if mixed:
                        e.shard_class_b(pb[r], pb[r + 1], k, np.asarray(h, dtype=np.uint64), canonical=canonical)
                        n = e.shard_sort_range_b(k, db[r], db[r + 1], rest_all, runs_all, canonical=canonical)
                    else:
                        n = e.shard_sort_range(k, db[r], db[r + 1], canonical=canonical)
                    e.materialize_keys()
                    u = e.unique_count_only()
                    rep = e.profile_report() if last else None
                    e.profile_enable(False)
                    return n, u, rep
                ms, (n, u, rep) = best_of(rank, args.reps, e.sync)
                extra.append({"device_ms": round(ms, 2), "collective_ms": round(coll, 3), "kmers": int(n)})
                record(ms + coll, rep)
                uniq += u
                kept += n
        else:
            import torch

            dev = torch.device("cuda", 0)
            so = not args.keys and not canonical and k <= 32 and e.is_acgt()  # (as ShardedKmerSort)
            wire = 4 if so else 12  # bytes per k-mer over xGMI
            sends, hists, part_ms = [], [], []
            for r in range(world):
                cap = pb[r + 1] - pb[r] + 64
                sk = None if so else torch.empty(cap, dtype=torch.int64, device=dev)
                sv = torch.empty(cap, dtype=torch.int32, device=dev)
                ms, (hist, n) = best_of(lambda _l, r=r, sk=sk, sv=sv: e.shard_partition(
                    pb[r], pb[r + 1], k, sk, sv, canonical=canonical, starts_only=so), args.reps, e.sync)
                sends.append((sk, sv))
                hists.append(np.asarray(hist, dtype=np.int64))
                part_ms.append(ms)
            H = np.stack(hists)
            bb = D.split_buckets(H.sum(axis=0), world)
            to = np.stack([[int(H[s, bb[d]:bb[d + 1]].sum()) for d in range(world)] for s in range(world)])
            for r in range(world):
                parts_k, parts_v = [], []
                for s in range(world):
                    lo = int(H[s, :bb[r]].sum())
                    if not so:
                        parts_k.append(sends[s][0][lo:lo + to[s, r]])
                    parts_v.append(sends[s][1][lo:lo + to[s, r]])
                R = int(to[:, r].sum())
                rk = None if so else torch.cat(parts_k + [torch.empty(64, dtype=torch.int64, device=dev)])
                rv = torch.cat(parts_v + [torch.empty(64, dtype=torch.int32, device=dev)])
                off, ln, bk = D.receive_pieces(H, bb[r], bb[r + 1], list(to[:, r]))
                torch.cuda.synchronize()

                def rank(last, r=r, rk=rk, rv=rv, R=R, off=off, ln=ln, bk=bk):
                    e.profile_enable(last)
                    e.shard_sort(rk, rv, R, k, off, ln, bk, canonical=canonical, starts_only=so)
                    e.materialize_keys()
                    u = e.unique_count_only()
                    rep = e.profile_report() if last else None
                    e.profile_enable(False)
                    return u, rep
                ms, (u, rep) = best_of(rank, args.reps, e.sync)
                peers = [d for d in range(world) if d != r]
                x_bytes = wire * max([int(to[r, d]) for d in peers] + [int(to[s, r]) for s in peers] + [0])
                x_ms = x_bytes / (LINK_GBS * 1e9) * 1e3
                extra.append({"partition_ms": round(part_ms[r], 2), "sort_ms": round(ms, 2),
                              "exchange_link_bound_ms": round(x_ms, 2),
                              "sent_gb": round(wire * (int(to[r].sum()) - int(to[r, r])) / 1e9, 3),
                              "wire_bytes_per_kmer": wire})
                record(part_ms[r] + x_ms + ms, rep)
                uniq += u
                kept += R
                del rk, rv
        assert kept == total, (kept, total)  # every k-mer on exactly one rank
        worst = max(per_rank)
        line = {"world": world, "per_rank_ms": per_rank, "max_rank_ms": worst,
                "mean_rank_ms": round(float(np.mean(per_rank)), 2),
                "kmers_per_s": round(total / (worst * 1e-3), 1),
                "speedup_vs_single": round(single_ms / worst, 2), "unique": uniq,
                "slowest_rank_stages_ms": stages}
        # the stages where ranks differ most (max - min over ranks > 0.2 ms)
        names = sorted({n for st in all_stages for n in st})
        spread = {n: [st.get(n, 0.0) for st in all_stages] for n in names}
        line["stage_spread_ms"] = {n: v for n, v in spread.items() if max(v) - min(v) > 0.2}
        if extra:
            line["ranks"] = extra
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
