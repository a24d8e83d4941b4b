"""Throughput of the SURVEY §8(f) rows around the sort, through the host API (genome_kmers), on one
GPU.  The default bench (bench.py) measures the sort path; this tool measures what sits either side
of it, at sizes that finish in about a minute:

  f1  filtered counts and group histograms on the device (kmers.py:454-648, 994-1178): a k = 31
      sort of a GRCh38-shaped genome, then get_kmer_count / get_kmer_group_counts with the
      reference's filter generators (no ambiguous bases, GC window, homopolymer) and get_kmers
  f2  FASTA -> sba ingestion (sequence_collection.py:476-576): a FASTA file of the same genome
      (60-column lines, 24 records) loaded by SequenceCollection(fasta_file_path=...)
  f3  variable-length mode (max_kmer_len=None, the Kmers default; kmers.py:306-397, 656-664):
      prefix doubling over every suffix of a random genome, and a bounded min < max sort
  f4  location info (kmers.py:1180-1264): get_kmers(kmer_info_to_yield="full")

Every query is timed twice (the first one also builds lazily allocated device state) and the
better time is reported; a sort is timed on a fresh object after a warm-up sort of another.
Parity for these rows is tested elsewhere (tests/test_gpu_*.py against the oracle and the
reference's fixtures); here each row carries a cheap self-consistency check.
The reference's published CPU rates, where SURVEY.md §8 quotes them, are listed for context.

usage (GPU box):  python tools/bench_next.py [--scale 3] [--vl-len 100000000] > gpurun_out/bench_next.json
"""
import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "genome-kmers_amd"))

import genome_kmers.kmers as gk  # noqa: E402
from genome_kmers import synthetic  # noqa: E402
from genome_kmers.sequence_collection import SequenceCollection  # noqa: E402


def log(msg):
    print(f"[bench_next {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def best_of(fn, reps=2):
    best, out = None, None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return best, out


def fresh_sort(make):
    """Time sort() on a fresh Kmers object, after a warm-up sort of another one (a second sort()
    of the same object would find the engine's order already in place)."""
    warm = make()
    warm.sort()
    del warm
    km = make()
    t0 = time.perf_counter()
    km.sort()
    km._engine.sync()  # sort() returns with the last kernels possibly still queued
    return time.perf_counter() - t0, km


def collection(sba, seg):
    """A SequenceCollection over an existing sba (the reference's attribute layout)."""
    sc = SequenceCollection()
    sc.forward_sba = sba
    sc._forward_sba_seg_starts = np.asarray(seg, dtype=np.uint32)
    sc.forward_record_names = [f"chr{i + 1}" for i in range(len(seg))]
    sc._strands_loaded = "forward"
    return sc


def write_fasta(path, sba, seg, width=60):
    """The records of sba as FASTA, `width` bases per line."""
    ends = list(np.asarray(seg[1:], dtype=np.int64) - 1) + [sba.size]
    with open(path, "wb") as f:
        for r, (s, e) in enumerate(zip(seg, ends)):
            rec = sba[int(s):int(e)]
            n = rec.size
            full = n // width
            body = np.empty(full * (width + 1), dtype=np.uint8)
            v = body.reshape(full, width + 1)
            v[:, :width] = rec[:full * width].reshape(full, width)
            v[:, width] = ord("\n")
            f.write(f">chr{r + 1} surrogate record {r + 1}\n".encode())
            f.write(body.tobytes())
            if n > full * width:
                f.write(rec[full * width:].tobytes() + b"\n")


def row(name, **kw):
    d = {"row": name, **kw}
    print(json.dumps(d), flush=True)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=3.0, help="GRCh38 contig lengths divided by this")
    ap.add_argument("--vl-len", type=int, default=100_000_000, help="genome length of the variable-length rows")
    ap.add_argument("--skip", default="", help="comma-separated rows to skip (f1,f2,f3,f4)")
    args = ap.parse_args()
    skip = set(filter(None, args.skip.split(",")))

    lengths = [max(1000, int(x / args.scale)) for x in synthetic.GRCH38_LENGTHS]
    log(f"GRCh38 surrogate at 1/{args.scale:g}: generating")
    sba, seg = synthetic.grch38_surrogate(2, lengths)
    L = int(sba.size)

    if "f2" not in skip:
        with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
            fa = Path(td) / "genome.fa"
            write_fasta(fa, sba, seg)
            size = fa.stat().st_size
            log(f"f2: FASTA of {size / 1e9:.2f} GB written")
            t, sc2 = best_of(lambda: SequenceCollection(fasta_file_path=fa))
            ok = bool(np.array_equal(sc2.forward_sba, sba))
            row("f2_fasta_ingest", seconds=round(t, 3), fasta_bytes=size, bases=L,
                gb_per_s=round(size / t / 1e9, 2), s_per_1e8_bases=round(t / L * 1e8, 3),
                reference_s_per_1e8_bases=2.45, reference_source="docs/development.rst:252 (SURVEY §8a1)",
                threads=os.environ.get("OMP_NUM_THREADS", "default"), sba_matches_generator=ok)
            del sc2

    sc = collection(sba, seg)
    if "f1" not in skip or "f4" not in skip:
        t, km = fresh_sort(lambda: gk.Kmers(sc, min_kmer_len=31, max_kmer_len=31))
        n = len(km)
        row("sort_k31_for_f1", seconds=round(t, 3), kmers=n, kmers_per_s=round(n / t, 1),
            note="host API sort() incl. its host round trips; bench.py times the device path")

    if "f1" not in skip:
        filters = {
            "no_ambiguous_bases": gk.gen_no_ambiguous_bases_filter(31),
            "gc_0.4_0.6": gk.gen_kmer_gc_content_filter_func(0.4, 0.6, 31),
            "homopolymer_le5": gk.gen_kmer_homopolymer_filter_func(5, 31),
            "keep_all": gk.kmer_filter_keep_all,
        }
        for fname, filt in filters.items():
            t, (hist, total) = best_of(lambda: km.get_kmer_group_counts(31, kmer_filter_func=filt,
                                                                        max_counts_bin=10000))
            hist = np.asarray(hist)
            consistent = bool(hist[-1] != 0 or int((np.arange(hist.size) * hist).sum()) == int(total))
            row("f1_group_counts", filter=fname, seconds=round(t, 4), kmers=n, kmers_per_s=round(n / t, 1),
                total=int(total), groups=int(hist.sum()), hist_total_consistent=consistent)
        t, cnt = best_of(lambda: km.get_kmer_count(31, kmer_filter_func=filters["no_ambiguous_bases"],
                                                   min_group_size=2))
        row("f1_kmer_count", filter="no_ambiguous_bases", min_group_size=2, seconds=round(t, 4), kmers=n,
            kmers_per_s=round(n / t, 1), count=int(cnt))
        t, got = best_of(lambda: sum(1 for _ in km.get_kmers(31, min_group_size=2, yield_first_n=1)))
        row("f1_get_kmers_minimum", min_group_size=2, yield_first_n=1, seconds=round(t, 4), kmers=n,
            kmers_per_s=round(n / t, 1), groups_yielded=int(got))

    if "f4" not in skip:
        t, got = best_of(lambda: sum(1 for _ in km.get_kmers(31, min_group_size=50, kmer_info_to_yield="full")))
        row("f4_get_kmers_full", min_group_size=50, seconds=round(t, 4), kmers=n, rows_yielded=int(got),
            rows_per_s=round(got / t, 1) if t > 0 else None)

    if "f1" not in skip or "f4" not in skip:
        del km

    if "f3" not in skip:
        vl = synthetic.random_bases(args.vl_len, 42)
        sc3 = collection(vl, [0])
        for mn, mx in ((1, None), (20, 40)):
            t, km3 = fresh_sort(lambda: gk.Kmers(sc3, min_kmer_len=mn, max_kmer_len=mx))
            n3 = len(km3)
            st = np.asarray(km3.kmer_sba_start_indices)
            # sampled order check: adjacent sorted suffixes compare non-decreasing (bytes, capped at mx)
            rng = np.random.default_rng(0)
            idx = rng.integers(0, n3 - 1, 2000)
            cap = 64 if mx is None else mx
            ok = all(bytes(vl[int(st[i]):int(st[i]) + cap]) <= bytes(vl[int(st[i + 1]):int(st[i + 1]) + cap])
                     for i in idx)
            row("f3_variable_length_sort", min_kmer_len=mn, max_kmer_len=mx, seconds=round(t, 3), kmers=n3,
                kmers_per_s=round(n3 / t, 1), sampled_adjacent_order_ok=ok,
                note="first 64 bytes compared for max_kmer_len=None (random genome: ties past 64 are absent)")
            del km3


if __name__ == "__main__":
    main()
