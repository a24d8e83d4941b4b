"""Headline benchmark: sorted 31-mers/s on a 3.1 Gb synthetic genome (BASELINE.json config C3).

One step = the hot path over the whole genome with the sequence byte array already in HBM:
enumerate -> encode (2-bit keys) -> stable MSD radix sort -> unique k-mers + multiplicities.
`value` is measured at the DEVICE boundary (the bench contract: inputs resident in HBM when the
timed region starts); the step ends with the whole product resident in HBM -- sorted start
indices, sorted keys, and per distinct k-mer its first sorted index and multiplicity.  The
end-to-end boundary of BASELINE.md section 3 is reported beside it: `value_e2e` is one wall-clock
interval from the sba in pinned host memory to the product in HBM (gk_set_sequence's transfer --
2-bit packed chunks and raw DMA chunks -- then one step), and the D2H of the sorted start indices
is reported apart.
Timed with a barrier + device synchronisation on both sides, max over ranks.

N = 1: the genome on one MI355X.  N > 1 (torch.distributed, one rank per GPU), total work fixed,
"scaling": "strong".  Every rank holds the whole sequence byte array (1 B per k-mer) and owns one
contiguous range of top key digits (genome_kmers.distributed):
  --exchange range (default): the digit ranges come from a 32 KiB all-reduce of per-rank 12-bit digit
      histograms; each rank re-derives its own k-mers from the whole sequence and sorts them --
      no k-mer crosses xGMI;
  --exchange a2a: each rank encodes its position share and the k-mers go to their owners in ONE
      all-to-all over RCCL (12 B per k-mer), then each rank sorts what it received.

Also reported: the dominant kernel's roofline (HIP events on the engine's stream) and the CPU
baseline -- the reference algorithm (numba-quicksort restatement, oracle/) on a bounded sample.
"""

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "genome-kmers_amd"))
sys.path.insert(0, str(ROOT))

METRIC = "sorted 31-mers/sec end-to-end on 3.1 Gb synthetic genome; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
# BASELINE.md section 3's byte model of the whole step: an 8-pass LSD sort of 8-byte keys with a
# 4-byte payload -- read 1 (sequence) + 8 (histogram) + 8 x 12 = 105 B per 31-mer, total 201 B
BASELINE_READ_B, BASELINE_TOTAL_B = 105, 201
# the wave-local finishing kernel's instantiation (gkm_msd.hip: msd_wave_kernel<I, waves/SIMD, keys>)
WAVE8_KERNEL = "msd_wave_kernel<8,4,true,9>"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=("c3", "c4", "c5", "ref_profile"), default="c3",
                    help="c3: the headline (3.1 Gb single contig, k=31); c4: GRCh38-shaped surrogate (24 "
                         "contigs, ~5%% N, diverged repeats), k=31; c5: the same genome, k=63, canonical; "
                         "ref_profile: the reference's own Kmers.sort profiling workload (tools/run_profiling.py "
                         "kmers_sort 'large': 1e8 bases in 10 contigs, min_kmer_len=1, --max-kmer-len 20 or none)")
    ap.add_argument("--max-kmer-len", default="20", help="ref_profile: max_kmer_len (an integer, or 'none')")
    ap.add_argument("--ref-bases", type=int, default=100_000_000, help="ref_profile: total sequence length")
    ap.add_argument("--genome-len", type=int, default=None, help="c3 genome length (default 3.1e9)")
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--cpu-sample", type=int, default=4_000_000,
                    help="k-mers in the CPU-baseline sample (starts spread over the whole genome: ~15 s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-boundary", action="store_true",
                    help="skip the transfers either side of the device boundary and the end-to-end interval "
                         "(profiler counter passes and A/B runs only)")
    ap.add_argument("--e2e-reps", type=int, default=5, help="end-to-end intervals per source (median reported)")
    ap.add_argument("--sharded", action="store_true",
                    help="use the multi-GPU path even at N = 1 (exercises it on one GPU)")
    ap.add_argument("--exchange", choices=("range", "a2a"), default="range",
                    help="multi-GPU scheme: key ranges re-derived from the resident sequence (no k-mer "
                         "exchange) or one all-to-all of the encoded k-mers")
    ap.add_argument("--opt", action="append", default=[], metavar="GKM_NAME=VALUE",
                    help="a libgkm test/tuning override (gk_set_option), for A/B runs; repeatable")
    ap.add_argument("--traffic", type=str, default=str(ROOT / "profiles" / "traffic_latest.json"),
                    help="per-launch HBM bytes of the dominant kernel from rocprofv3 --pmc (if present)")
    return ap.parse_args()


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(sba: np.ndarray, k: int, sample: int, n_full: int) -> dict:
    """Reference algorithm (Kmers.sort: numba quicksort + byte comparator with validation,
    kmers.py:1624-1731) restated in C (oracle/gk_oracle.c), 1 thread (the reference is
    single-threaded, kmers.py:1644-1648), per BASELINE.md section 2:
      C1 in full (10 kb, np.random.seed(42) random ACGT as profiling.get_random_seq, k = 5);
      C2 in full (the 4,641,652 bp surrogate, k = 31);
      `value`: a bounded sample of this run's workload in the DRAM regime of the full run --
      `sample` k-mers whose starts are spread evenly over the WHOLE genome (every comparison reads
      two windows anywhere in the 3.1 GB sba, as the full sort's do), and its N log2 N
      extrapolation to the full workload, labelled as such;
      context: `sample` CONSECUTIVE k-mers (a few-MB window: cache-resident, faster), and
      the 1e8 / 3e8-base prefix runs measured outside the bench's budget."""
    from genome_kmers import synthetic
    from oracle import oracle

    def timed(seq, starts, kk):
        t0 = time.perf_counter()
        oracle.quicksort(seq, starts, kk, kk)
        return len(starts), time.perf_counter() - t0

    c1_seq = np.frombuffer(b"ATGC", dtype=np.uint8)[np.random.RandomState(42).randint(0, 4, 10_000)]
    n1, t1 = timed(c1_seq, np.arange(10_000 - 5 + 1, dtype=np.uint32), 5)
    c2 = synthetic.c2_surrogate()[0]
    n2, t2 = timed(c2, np.arange(len(c2) - 31 + 1, dtype=np.uint32), 31)
    # DRAM regime: starts spread over the whole genome (the genome is one N-free contig at C3;
    # a start whose window holds '$' or N is skipped)
    span = len(sba) - k + 1
    spread = (np.arange(sample, dtype=np.uint64) * (span // sample)).astype(np.uint32)
    if np.any(sba == 36) or np.any(sba == ord("N")):
        bad = np.zeros(len(sba) + 1, dtype=np.int64)
        bad[1:] = np.cumsum((sba == 36) | (sba == ord("N")))
        spread = spread[bad[spread.astype(np.int64) + k] == bad[spread.astype(np.int64)]]
    ns, dt = timed(sba, spread, k)
    t_full = dt * (n_full * np.log2(n_full)) / (ns * np.log2(ns))
    # context: consecutive k-mers of a contig-free window
    at = len(sba) // 3
    sub = np.ascontiguousarray(sba[at: at + sample + k - 1])
    if np.any(sub == 36) or np.any(sub == ord("N")):
        sub = np.ascontiguousarray(sba[: sample + k - 1])
    nc, tc = timed(sub, np.arange(len(sub) - k + 1, dtype=np.uint32), k)
    # BASELINE.md section 2's prefix runs (1e8 / 3e8 bases of the C3 genome), measured outside the
    # bench's budget by tools/cpu_baseline_prefixes.py on a GPU box's host (~10 min)
    prefixes = None
    pre_path = ROOT / "profiles" / "r4" / "cpu_baseline_prefixes.json"
    if not pre_path.exists():
        pre_path = ROOT / "profiles" / "r3" / "cpu_baseline_prefixes.json"
    try:
        with open(pre_path) as fh:
            pre = json.load(fh)
        prefixes = {"source": str(pre_path.relative_to(ROOT)), "cpu_model": pre["cpu_model"],
                    "genome": pre.get("genome", "numpy PCG64 seed 42 (round 3)"),
                    "runs": pre["prefixes"], "full_workload": pre["full_workload"]}
    except (OSError, ValueError, KeyError):
        pass
    return {"value": ns / dt, "unit": "k-mers/s", "cores": 1, "kind": "port",
            "sample": f"{ns:,} {k}-mers with starts spread evenly over the whole {len(sba):,}-base genome (the "
                      f"full sort's DRAM-miss regime), numba-quicksort restatement with validate_kmers, gcc -O3, "
                      f"1 thread; {dt:.1f} s",
            "cpu_model": _cpu_model(), "cores_on_box": os.cpu_count(),
            "c1": {"kmers": n1, "seconds": round(t1, 4), "kmers_per_s": round(n1 / t1, 1)},
            "c2": {"kmers": n2, "seconds": round(t2, 3), "kmers_per_s": round(n2 / t2, 1)},
            "consecutive_sample": {"kmers": nc, "seconds": round(tc, 2), "kmers_per_s": round(nc / tc, 1),
                                   "note": "consecutive k-mers of one window: cache-resident, not the full "
                                           "run's regime (context only)"},
            "full_workload_extrapolated": {"kmers": n_full, "seconds": round(t_full, 1),
                                           "kmers_per_s": round(n_full / t_full, 1),
                                           "method": "spread-sample time x (N log2 N) / (n log2 n); extrapolated, "
                                                     "not measured"},
            "prefix_runs": prefixes}


def window_check(eng, sba: np.ndarray, k: int, canonical: bool, width: int = 2048) -> int:
    """Cheap self-check of the sorted output after the timed steps (no oracle: plain numpy over the
    sba): windows of the sorted starts -- at the ends, the middle and past 2^31 -- must be
    non-decreasing by k-mer bytes (canonical: min with the reverse complement), with equal k-mers
    in ascending start order.  Returns the number of k-mers checked."""
    n = eng.n
    comp = np.arange(256, dtype=np.uint8)
    for a, b in zip(b"ACGTRYSWKMBDHVN$", b"TGCAYRSWMKVHDBN$"):
        comp[a] = b
    offs = sorted({0, max(n // 2 - width // 2, 0), max(n - width, 0)} | ({2**31 + 1} if n > 2**31 + width else set()))
    checked = 0
    for off in offs:
        w = eng.start_range(off, min(width, n - off)).astype(np.int64)
        rows = sba[w[:, None] + np.arange(k)[None, :]]
        if canonical:
            rc = comp[rows[:, ::-1]]
            d = rows != rc
            first = d.argmax(axis=1)
            r = np.arange(len(w))
            use_rc = d.any(axis=1) & (rc[r, first] < rows[r, first])
            rows = np.where(use_rc[:, None], rc, rows)
        d = rows[1:] != rows[:-1]
        first = d.argmax(axis=1)
        r = np.arange(len(w) - 1)
        tie = ~d.any(axis=1)
        ok = np.where(tie, w[1:] > w[:-1], rows[1:][r, first] > rows[:-1][r, first])
        if not ok.all():
            raise SystemExit(f"bench self-check: sorted order broken at index {off + int(np.argmin(ok))}")
        checked += len(w)
    return checked


def transfer_times(torch, eng, sba, seg, log, reps: int = 3) -> dict:
    """The transfers either side of the device boundary, after the timed
    steps, best of reps: the D2H of the sorted start indices into pinned host memory; gk_set_sequence
    (gkm_xfer.hip) from pinned host memory (packed chunks from the front, raw DMA from the back)
    and from the caller's pageable numpy sba (packed only) until the sba is resident; and, for
    context, a plain H2D of the ASCII sba from pinned host memory (one unpacked copy)."""
    n = eng.n
    out = {}
    host = torch.empty(max(n, 1), dtype=torch.int32).pin_memory().numpy().view(np.uint32)
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        eng.copy_starts(host[:n])
        best = min(best, time.perf_counter() - t0)
    out["d2h_starts_ms"] = round(best * 1e3, 2)
    out["d2h_starts_gbs"] = round(4 * n / best / 1e9, 1)
    del host
    best = float("inf")
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.set_sequence(sba, seg)
        eng.sync()
        best = min(best, time.perf_counter() - t0)
    out["set_sequence_pageable_ms"] = round(best * 1e3, 2)
    pinned = torch.empty(len(sba), dtype=torch.uint8).pin_memory()
    pinned.numpy()[:] = sba
    best = float("inf")
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.set_sequence(pinned.numpy(), seg)
        eng.sync()
        best = min(best, time.perf_counter() - t0)
    out["set_sequence_ms"] = round(best * 1e3, 2)
    out["set_sequence_gbs"] = round(len(sba) / best / 1e9, 1)
    dev = torch.empty(len(sba), dtype=torch.uint8, device="cuda")
    best = float("inf")
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev.copy_(pinned, non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    del dev, pinned
    out["h2d_ascii_pinned_ms"] = round(best * 1e3, 2)
    out["h2d_ascii_pinned_gbs"] = round(len(sba) / best / 1e9, 1)
    log(f"transfers: {out}")
    return out


def end_to_end(torch, eng, sba, seg, step, log, reps: int = 5, hint_k: int = 0) -> dict:
    """BASELINE.md section 3's end-to-end boundary, measured as one wall-clock interval: from the sba
    in pinned host memory (the contract's source) to the whole product resident in HBM --
    gk_set_sequence (the sequence packed to 2 bits on the host threads, copied in chunks, unpacked
    on the device) followed by one step, device synchronised.  The MEDIAN of `reps` intervals (every
    interval is listed).  hint_k: the sort hint (gk_sort_hint) is set, so the transfer also runs the
    sort's first pass (L0) over the regions of the sequence as they land -- what Kmers(sc, k, k)
    does -- and the same interval without the hint is reported beside it.  The same from the
    caller's pageable numpy array is reported too."""
    pinned = torch.empty(len(sba), dtype=torch.uint8).pin_memory()
    pinned.numpy()[:] = sba
    out = {}
    runs = [("pinned", pinned.numpy(), hint_k), ("pageable", sba, hint_k)]
    if hint_k:
        runs.append(("pinned_nohint", pinned.numpy(), 0))
    for name, src, hk in runs:
        eng.sort_hint(hk)
        tot, sets = [], []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.set_sequence(src, seg)
            t1 = time.perf_counter()
            step()
            eng.sync()
            t2 = time.perf_counter()
            tot.append((t2 - t0) * 1e3)
            sets.append((t1 - t0) * 1e3)
        out[f"e2e_{name}_ms"] = round(float(np.median(tot)), 2)
        out[f"e2e_{name}_reps_ms"] = [round(x, 2) for x in tot]
        out[f"set_sequence_host_{name}_ms"] = round(float(np.median(sets)), 2)
    eng.sort_hint(0)
    del pinned
    out["sort_hint_k"] = hint_k
    out["e2e_ms"] = out["e2e_pinned_ms"]
    out["e2e_stat"] = f"median of {reps}"
    log(f"end to end: {out}")
    return out


def load_traffic(path: str, kernel: str):
    """(HBM bytes per launch, source) of `kernel` (an instantiation prefix such as
    "msd_pipe_kernel<1024,11,8,4") from a tools/pmc_traffic.py summary -- rocprofv3 --pmc passes
    of FETCH_SIZE and WRITE_SIZE over this same bench command on a builder's box (a bench run
    cannot read PMC counters itself); (None, reason) when the file has no such kernel."""
    try:
        with open(path) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None, f"{path}: not found"
    rel = os.path.relpath(path, ROOT)
    want = kernel.replace(" ", "").rstrip(">")
    for name, rec in t.items():
        if not name.startswith("_") and "<" in name and name.startswith(want):
            return rec.get("hbm_bytes_max_launch"), f"{rel} ({t.get('_label', '')}; {t.get('_convention', '')})"
    return None, f"{rel}: no {kernel} record"


def ref_profile_sba(total: int, contigs: int = 10, seed: int = 42):
    """profiling.get_random_seq_list(total, contigs) after np.random.seed(seed) (profiling.py:30-60):
    contigs of total // contigs bases (the last takes the rest), drawn one after another from the
    same stream, joined by '$' as SequenceCollection does (sequence_collection.py:663-726)."""
    from genome_kmers import _native

    bases = _native.reference_random_bases(total, seed)
    avg = total // contigs
    cuts = [i * avg for i in range(contigs)] + [total]
    sba = np.empty(total + contigs - 1, dtype=np.uint8)
    seg = np.empty(contigs, dtype=np.uint32)
    at = 0
    for i in range(contigs):
        piece = bases[cuts[i]:cuts[i + 1]]
        seg[i] = at
        sba[at:at + len(piece)] = piece
        at += len(piece)
        if i + 1 < contigs:
            sba[at] = 36
            at += 1
    return sba, seg


def order_check(eng, sba: np.ndarray, max_len, width: int = 2048) -> int:
    """Self-check of a variable-length / suffix sort (no oracle): windows of the sorted starts are
    non-decreasing by their k-mers -- bytes up to '$' (or the end), capped at max_len -- with equal
    k-mers in ascending start order."""
    n = eng.n
    cap = max_len if max_len is not None else 1 << 62

    def kmer(s):
        w = 64
        while True:
            b = bytes(sba[s:s + min(w, cap)]).split(b"$")[0]
            if len(b) < min(w, cap) or w >= cap or s + w >= len(sba):
                return b
            w *= 4

    checked = 0
    for off in sorted({0, max(n // 2 - width // 2, 0), max(n - width, 0)}):
        w = eng.start_range(off, min(width, n - off)).tolist()
        prev = kmer(w[0])
        for a, b in zip(w, w[1:]):
            cur = kmer(b)
            if cur < prev or (cur == prev and b < a):
                raise SystemExit(f"bench self-check: sorted order broken near index {off}")
            prev = cur
        checked += len(w)
    return checked


def run_ref_profile(args, torch, result_out, log):
    """The reference's own profiled sort workload (tools/run_profiling.py:226-236, profiling.py:367-448):
    Kmers(min_kmer_len=1, max_kmer_len=M).sort() over 1e8 bases in 10 contigs, seed 42.  A step is
    enumerate + sort, the call the reference times (run_kmers_sort).  M = 20: bounded variable-length
    keys (2-bit padded symbols + length, 45 bits) through the MSD levels over the keys (the LSD onesweep
    with GKM_SORT_KEYS_LSD=1); M = None (the Kmers default): prefix doubling."""
    from genome_kmers import _native
    from oracle import oracle

    M = None if str(args.max_kmer_len).lower() == "none" else int(args.max_kmer_len)
    sba, seg = ref_profile_sba(args.ref_bases)
    eng = _native.Engine(0)
    eng.set_sequence(sba, seg)
    eng.sync()
    n = eng.enumerate(1)

    def step():
        eng.enumerate(1)
        eng.sort(M)

    for _ in range(args.warmup):
        step()
    eng.sync()
    eng.profile_enable(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    report = eng.profile_report()
    eng.profile_enable(False)
    checked = order_check(eng, sba, M)
    words, bits, _ = eng.key_layout()
    stages = {name: round(v["total_ms"] / args.steps, 3) for name, v in report.items()}
    # the whole step against the HBM peak: the algorithmic bytes of every priced stage per step over
    # the step's wall time (the dominant kernel's `frac` is one kernel; this is all of them, and the
    # step's unpriced remainder -- scans, classify, host round trips -- counts as time)
    step_bytes = sum(stage_bytes(n, v) for n, v in report.items() if v.get("total_ms", 0) > 0) / args.steps
    step_frac = step_bytes / (ms_per_step * 1e-3) / (HBM_PEAK_GBS * 1e9)
    msd = "radix_pass" not in report and any(k.startswith("msd_") for k in report)
    if not msd:
        # dominant kernel: the LSD onesweep pass (every radix_pass launch: keys W words + start in and out)
        rp = report.get("radix_pass", {"count": 0, "total_ms": 0.0, "units": 0})
        per_unit = 2 * (8 * max(words, 1) + 4)
        kernel = f"onesweep_kernel (W = {max(words, 1)}; radix_pass: one stable 8-bit LSD pass with decoupled look-back)"
    else:
        # the MSD levels over the keys (sort_keys, gkm_sort.hip): the stage with the most time among
        # the level partitions and the finishing kernels, priced as in the C3 model (run())
        compact_in = any(k.startswith("msd_pass_l") and k.endswith("c") for k in report)
        pairs_in = any(k.startswith("msd_pass_l") and k.endswith("p") for k in report)

        def unit_bytes(name):
            if name.startswith("msd_pass_l") and name.endswith("c"):
                return 19 if pairs_in else 21
            if name.startswith("msd_pass_l") and name.endswith("p"):
                return 23
            if name.startswith("msd_pass_l"):
                return 24
            if name.startswith("msd_local"):
                return 22 if compact_in else 25
            return 0

        timed = {k: v for k, v in report.items() if unit_bytes(k) and v["total_ms"] > 0 and v.get("units", 0)}
        dom = max(timed, key=lambda k: timed[k]["total_ms"]) if timed else None
        rp = timed.get(dom, {"count": 0, "total_ms": 0.0, "units": 0})
        per_unit = unit_bytes(dom) if dom else 0
        kernel = (f"{WAVE8_KERNEL if dom == 'msd_local_wave8' else 'msd_pipe_kernel<1024,11,R>'} ({dom}: "
                  f"MSD levels over the keys in memory)")
    avg_ms = rp["total_ms"] / max(rp["count"], 1)
    units = rp["units"] / max(rp["count"], 1)
    achieved = per_unit * units / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    cpu = None
    if not args.no_cpu_baseline:
        # DRAM regime: 2M starts spread over the whole sba (every position outside '$' is a start)
        valid = np.flatnonzero(sba != 36).astype(np.uint32)
        sample = valid[:: max(1, len(valid) // 2_000_000)]
        t1 = time.perf_counter()
        oracle.quicksort(sba, sample, 1, M)
        tc = time.perf_counter() - t1
        ns = len(sample)
        t_full = tc * (n * np.log2(n)) / (ns * np.log2(ns))
        cpu = {"value": ns / tc, "unit": "k-mers/s", "cores": 1, "kind": "port",
               "sample": f"{ns:,} starts spread over the whole {len(sba):,}-byte sba, numba-quicksort restatement "
                         f"of Kmers.sort (min_kmer_len=1, max_kmer_len={M}) with validate_kmers, gcc -O3, 1 thread; "
                         f"{tc:.1f} s",
               "cpu_model": _cpu_model(), "cores_on_box": os.cpu_count(),
               "full_workload_extrapolated": {"kmers": n, "seconds": round(t_full, 1),
                                              "kmers_per_s": round(n / t_full, 1),
                                              "method": "sample time x (N log2 N) / (n log2 n); extrapolated, not "
                                                        "measured"}}
    line = {
        "metric": f"Kmers.sort() k-mers/sec on the reference's profiling workload (run_profiling.py kmers_sort "
                  f"'large': {args.ref_bases:,} bases, 10 contigs, min_kmer_len=1, max_kmer_len={M})",
        "value": round(n * args.steps / dt, 1), "unit": "k-mers/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: profiling.get_random_seq_list(1e8, 10) after np.random.seed(42) (MT19937 stream, "
                "gk_reference_random_bases)",
        "boundary": "device: sba resident in HBM; step = enumerate + sort (the call the reference times); sorted "
                    "starts and keys (M=20) / ranks (M=None) resident at the end",
        "self_check": f"{checked:,} sorted k-mers in windows re-checked against the sba bytes",
        "config": {"workload": f"ref_profile: {args.ref_bases:,} bases in 10 contigs, min_kmer_len=1, "
                               f"max_kmer_len={M}", "kmers": n,
                   "sort_path": (("MSD levels over" if msd else "LSD onesweep over") + " (2-bit padded, length) keys")
                                if M is not None and bits else
                                ("prefix doubling: seed keys (MSD), then the tied groups by the rank of p + h"
                                 if msd else "prefix doubling (seed keys, then rank pairs, LSD)"),
                   "key_words": words, "key_bits": bits, "stages_ms_per_step": stages},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": kernel,
                     "avg_launch_ms": round(avg_ms, 4), "launches_per_step": round(rp["count"] / args.steps, 2),
                     "units_per_launch": int(units), "bytes_per_unit": per_unit},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), file=result_out, flush=True)


def main():
    args = parse()
    # the JSON line is the only thing on stdout: libraries (RCCL prints a banner at its first
    # collective) write to fd 1 as well, so fd 1 goes to stderr and the line to a saved copy
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dist = None
    if world > 1 or args.sharded:
        import torch.distributed as dist

        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29531")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), rank=rank, world_size=world)

    from genome_kmers import _native, synthetic

    for o in args.opt:
        name, _, v = o.partition("=")
        _native.options[name] = v
    if args.config == "ref_profile":
        if world != 1:
            raise SystemExit("--config ref_profile runs on one GPU")
        return run_ref_profile(args, torch, result_out,
                               lambda m: print(f"[bench] {m}", file=sys.stderr, flush=True))
    cfg = args.config
    k = args.k or (63 if cfg == "c5" else 31)
    canonical = cfg == "c5"
    seed = args.seed if args.seed is not None else (42 if cfg == "c3" else 2)
    if cfg == "c3":
        L = args.genome_len or 3_100_000_000
        sba, seg = synthetic.c3_genome(L, seed)
        workload = f"C3: {L:,}-base synthetic single-contig genome, k={k} (min=max={k})"
        data = (f"synthetic: the reference's profiling genome, profiling.get_random_seq({L}) after "
                f"np.random.seed({seed}) (MT19937 stream, made by gk_reference_random_bases)")
    else:
        sba, seg = synthetic.grch38_surrogate(seed)
        L = len(sba)
        workload = (f"{cfg.upper()}: GRCh38-shaped surrogate (24 contigs, {L:,} sba bytes), k={k}"
                    + (", canonical" if canonical else ""))
        data = (f"synthetic GRCh38 surrogate: contig lengths of GRCh38, random ACGT + ~5% N + diverged repeat "
                f"families, numpy PCG64 seed {seed} (no FASTA on the box)")

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    if world == 1 and not args.sharded:
        eng = _native.Engine(local)
        t0 = time.perf_counter()
        eng.set_sequence(sba, seg)
        eng.sync()
        h2d_ms = (time.perf_counter() - t0) * 1e3
        n_units = eng.enumerate(k)

        def step():
            eng.enumerate(k)
            eng.sort(k, canonical=canonical)
            eng.materialize_keys()  # a one-word sort wrote them; else re-encoded (timed either way)
            return eng.unique_count_only()  # group starts + multiplicities, resident in HBM
    else:
        from genome_kmers import distributed

        cls = distributed.KeyRangeKmerSort if args.exchange == "range" else distributed.ShardedKmerSort
        job = cls(sba, seg, k, rank, world, device=local, canonical=canonical)
        eng = job.engine
        h2d_ms = job.h2d_ms
        n_units = job.total_kmers

        def step():
            return job.run()

    def log(msg):
        print(f"[bench rank {rank}] {msg}", file=sys.stderr, flush=True)

    log(f"{cfg}: {n_units:,} k-mers, sba on the device; warmup")
    n_unique = None
    for i in range(args.warmup):
        n_unique = step()
        log(f"warmup step {i} done")
    barrier()
    eng.profile_enable(True)
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        n_unique = step()
        log(f"step {i} queued")
    eng.sync()
    barrier()
    dt = time.perf_counter() - t0
    report = eng.profile_report()
    eng.profile_enable(False)
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        u = torch.tensor([n_unique], dtype=torch.int64, device="cuda")
        dist.all_reduce(u)
        n_unique = int(u.item())

    ms_per_step = dt / args.steps * 1e3
    value = n_units * args.steps / dt

    # the product's boundary: self-check, then the transfers either side of the device boundary
    # (timing experiments of a stage's memory floor write wrong output on purpose: no check)
    checked = (0 if os.environ.get("GKM_EXP_WAVECOPY") or os.environ.get("GKM_EXP_L0")
               else window_check(eng, sba, k, canonical))
    if dist is not None:
        t = torch.tensor([job.local_kmers], dtype=torch.int64, device="cuda")
        dist.all_reduce(t)
        if int(t.item()) != n_units:
            raise SystemExit(f"bench self-check: ranks hold {int(t.item())} k-mers, expected {n_units}")
    e2e, e2e_ms = None, None
    if args.no_boundary:
        boundary = {"set_sequence_ms": None, "d2h_starts_ms": None}
    else:
        boundary = transfer_times(torch, eng, sba, seg, log)
    if args.no_boundary:
        pass
    elif dist is None:
        # the sort hint applies to the fixed-length forward sort of an ACGT sequence (C3; any number of
        # contigs since round 6 -- a non-ACGT sequence drops it as the transfer packs its first such byte)
        hint = k if (not canonical and 8 <= k <= 32) else 0
        e2e = end_to_end(torch, eng, sba, seg, step, log, args.e2e_reps, hint)
        e2e_ms = e2e["e2e_ms"]
    else:  # ranks: each loads the whole sba; the slowest transfer + the step (max over ranks)
        t = torch.tensor([boundary["set_sequence_ms"], boundary["d2h_starts_ms"]], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        boundary["set_sequence_ms"], boundary["d2h_starts_ms"] = round(float(t[0]), 2), round(float(t[1]), 2)
        e2e_ms = ms_per_step + boundary["set_sequence_ms"]
    value_e2e = n_units / (e2e_ms * 1e-3) if e2e_ms else None

    # per-stage algorithmic bytes per work unit (k-mer), DESIGN.md section 4.  The L0 passes read
    # the sequence: its resident 2-bit packed copy when gk_set_sequence left one (0.375 B per
    # position: a u64 of codes and a u32 of stop flags per 32 positions), else the ASCII bytes
    packed_in = eng.resident_packed()  # (an ACGT sba's L0, or the class-A L0 of a mixed one)
    seq_positions = L if dist is None or args.exchange == "range" else job.hi - job.lo
    seq_bytes = seq_positions * (0.375 if packed_in else 1.0)

    range_mode = dist is not None and args.exchange == "range"
    # the last global level was compact: the wave-local round reads 9 B per element, not 12; a
    # packed-pair level before it wrote 10 B (+ digit byte) per element, which the compact level reads
    compact_in = any(n.startswith("msd_pass_l") and n.endswith("c") for n in report)
    pairs_in = any(n.startswith("msd_pass_l") and n.endswith("p") for n in report)
    # the packed L0 (msd_pass_l0k): digit byte + packed pair + low start bits, 11 B per element out,
    # which the level behind it reads (11 B in instead of 12)
    l0_packed = "msd_pass_l0k" in report

    def stage_bytes(name, v):
        u = v.get("units", 0)
        if name == "msd_select_count":
            return u  # key-range shards: the whole sequence, 1 B per position
        if name == "msd_select":
            return seq_bytes * v["count"] + 13 * u  # the whole sequence in; kept (key, start, digit) out (units: kept)
        if name == "msd_l0_count":
            return seq_bytes * v["count"]  # the sequence in (per-tile digit counts out: negligible)
        if name == "histogram":
            return seq_bytes / max(world, 1) * v["count"]  # the rank's position share of the sequence
        if name == "msd_count_nd":
            return u  # 1 digit byte per element in
        if name == "msd_pass_l0" and not range_mode:
            return seq_bytes * v["count"] + 13 * u  # sequence bytes in, (key, start, next digit) out
        if name == "msd_pass_l0k" and not range_mode:
            return seq_bytes * v["count"] + 11 * u  # sequence bytes in, (digit byte, pair, low start bits) out
        if name.startswith("msd_pass_l") and name.endswith("c"):
            # compact level: (key, start) -- or a packed pair, 10 B -- in, (low bits | start) + next digit out
            return (19 if pairs_in else 21) * u
        if name.startswith("msd_pass_l") and name.endswith("p"):
            # packed-pair level: (key, start) -- or, behind the packed L0, its 11 B -- in, pair (10 B)
            # + next digit out
            return (22 if l0_packed and name == "msd_pass_l1p" else 23) * u
        if name.startswith("msd_pass_l"):
            return 24 * u  # (key 8 B, start 4 B) in and out
        if name.startswith("msd_local"):
            # (key 8 B, start 4 B) in -- or, behind a compact level, (low bits | start) 8 B + digit
            # byte 1 B; key, start and 1 head flag out
            return (22 if compact_in else 25) * u
        if name == "msd_count":
            return 8 * u
        if name == "unique_counts":
            return n_units * v["count"] + 8 * n_unique * v["count"]  # head flags in; start + count out
        return 0

    kernels = {}
    for name, v in report.items():
        b = stage_bytes(name, v)
        if b and v["total_ms"] > 0:
            kernels[name] = {"ms_per_launch": round(v["total_ms"] / v["count"], 4),
                             "gbs": round(b / (v["total_ms"] * 1e-3) / 1e9, 1)}
    # dominant kernel: the stage with the most time among the device kernels with a byte model
    # (the level partitions, the compact level, the L0 partition, the wave-local finishing kernel)
    wide = "msd_local_block32" in report  # the 11-bit L0 leaves ~5.9 K-key buckets for the 1024-thread class
    kinds = {"msd_pass_l0": (("msd0_wide_kernel<512,36,11,true>", "the 11-bit L0 partition, straight from the "
                              "sequence") if wide else
                             ("msd0_pipe_kernel<2,1024,24,7,true>", "the L0 partition, straight from the sequence")),
             "msd_pass_l0k": ("msd0_pipe_kernel<2,1024,24,7,true,false,false,true>",
                              "the L0 partition, straight from the sequence, packed output"),
             "msd_local_wave8": (WAVE8_KERNEL, "wave-local finishing of buckets <= 512"),
             "msd_local_block32": ("msd_local_kernel<1024,8,10>", "block-local finishing of buckets <= 8192")}
    timed = {n: v for n, v in report.items() if stage_bytes(n, v) and v["total_ms"] > 0 and
             (n in kinds or n.startswith("msd_pass_l"))}
    dom = max(timed, key=lambda n: timed[n]["total_ms"]) if timed else None
    rp = timed.get(dom, {"count": 0, "total_ms": 0.0, "units": 0})
    dom_bytes = stage_bytes(dom, rp) if dom else 0
    if dom in kinds:
        kdesc, what = kinds[dom]
    elif dom and dom.endswith("c"):
        kdesc, what = (("msd_pipe_kernel<1024,11,8,4,true,0,true>", "the compact last level's stable 8-bit partition "
                        "(packed-pair input)") if pairs_in else
                       ("msd_pipe_kernel<1024,11,8,4>", "the compact last level's stable 8-bit partition"))
    elif dom and dom.endswith("p"):
        kdesc, what = (("msd_pipe_kernel<1024,11,8,5,true,0,2>", "one stable 8-bit MSD partition pass reading the "
                        "packed L0 output and writing packed pairs") if l0_packed and dom == "msd_pass_l1p" else
                       ("msd_pipe_kernel<1024,11,8,5>", "one stable 8-bit MSD partition pass writing packed pairs"))
    else:
        kdesc, what = "msd_pipe_kernel<1024,11,8,0>", "one stable 8-bit MSD partition pass"
    avg_ms = rp["total_ms"] / max(rp["count"], 1)
    bytes_per_launch = dom_bytes / max(rp["count"], 1)
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    stages = {name: round(v["total_ms"] / args.steps, 3) for name, v in report.items()}
    # the whole step against the HBM peak: the algorithmic bytes of every priced stage per step over
    # the step's wall time (the dominant kernel's `frac` is one kernel; this is all of them, and the
    # step's unpriced remainder -- scans, classify, host round trips -- counts as time)
    step_bytes = sum(stage_bytes(n, v) for n, v in report.items() if v.get("total_ms", 0) > 0) / args.steps
    step_frac = step_bytes / (ms_per_step * 1e-3) / (HBM_PEAK_GBS * 1e9)
    traffic, traffic_src = load_traffic(args.traffic, kdesc)
    # BASELINE.md section 3, verbatim: the step's read roofline n * 105 B / t (device boundary and
    # end to end), and the total-traffic fraction n * 201 B / t -- a model of the whole step, beside
    # the dominant kernel's own byte model above
    t_dev, t_e2e = ms_per_step * 1e-3, (e2e_ms or float("nan")) * 1e-3
    base = {"baseline_read_frac": round(n_units * BASELINE_READ_B / t_dev / (HBM_PEAK_GBS * 1e9), 4),
            "baseline_read_frac_e2e": (round(n_units * BASELINE_READ_B / t_e2e / (HBM_PEAK_GBS * 1e9), 4)
                                       if e2e_ms else None),
            "baseline_total_frac": round(n_units * BASELINE_TOTAL_B / t_dev / (HBM_PEAK_GBS * 1e9), 4),
            "baseline_model": "BASELINE.md section 3: read 105 B, total 201 B per 31-mer (8-pass LSD model) / "
                              "ms_per_step (device) or e2e_ms (end to end) / 8 TB/s"}
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                "step_hbm_frac": round(step_frac, 4), "step_algorithmic_bytes": int(step_bytes),
                "step_model": "sum of every priced stage's algorithmic bytes (DESIGN.md section 4; the L0 "
                              "input priced as the " + ("0.375 B/position resident packed copy" if packed_in else
                                                        "1 B/position sequence bytes") +
                              ") per step / ms_per_step / 8 TB/s -- the measured whole-step HBM fraction, beside "
                              "BASELINE.md's 8-pass LSD model (baseline_read_frac)",
                **base,
                "kernel": f"{kdesc} ({dom}: {what})",
                "avg_launch_ms": round(avg_ms, 4), "algorithmic_bytes_per_launch": int(bytes_per_launch),
                "units_per_launch": int(rp["units"] / max(rp["count"], 1)),
                "bytes_per_unit": round(bytes_per_launch / max(rp["units"] / max(rp["count"], 1), 1), 2),
                "stages": kernels}

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(sba, k, args.cpu_sample, n_units)
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "k-mers/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u64",
            **({} if cfg == "c3" else {"metric": f"sorted {k}-mers/sec end-to-end on the GRCh38 surrogate"
                                                 + (" (canonical)" if canonical else "")}),
            "data": data,
            "boundary": "value: device (sba resident in HBM at the start; sorted starts, sorted keys, first index "
                        "+ multiplicity of every distinct k-mer resident in HBM at the end); value_e2e: one wall-clock "
                        "interval from the sba in pinned host memory to that product in HBM (gk_set_sequence's "
                        "packed / raw transfer + one step; BASELINE.md section 3); the D2H of the "
                        "sorted starts is reported apart (d2h_starts_ms)",
            "value_boundary": "device: the sba resident in HBM when the timed region starts (the bench contract)"
                              + ("; with it the 2-bit packed copy of the sequence (1.17 GB at C3) that "
                                 "gk_set_sequence's packed transfer writes beside the sba outside the timed region "
                                 "-- the L0 passes read it (0.375 B/position)" if packed_in else "") +
                              "; the end-to-end figure of BASELINE.md section 3, pinned host sba -> product in HBM "
                              "(transfer + packed copy + step), is value_e2e",
            "value_e2e": round(value_e2e, 1) if value_e2e else None, "e2e_ms": round(e2e_ms, 2) if e2e_ms else None,
            **({} if e2e is None else {"e2e": e2e}),
            "set_sequence_ms": boundary["set_sequence_ms"], "d2h_starts_ms": boundary["d2h_starts_ms"],
            "self_check": f"{checked:,} sorted k-mers in windows re-checked against the sba bytes",
            "config": {"workload": workload,
                       "genome_bases": L, "k": k, "kmers": n_units, "unique_kmers": n_unique,
                       "parallelism": ("1 GPU" if dist is None else
                                       f"key-range shards x{world}: whole sba per rank, 32 KiB RCCL all-reduce, "
                                       "no k-mer exchange" if args.exchange == "range" else
                                       f"position-range shards x{world} + 1 RCCL all-to-all of the k-mers"),
                       "first_set_sequence_ms": round(h2d_ms, 2), "transfers": boundary,
                       "stages_ms_per_step": stages},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), file=result_out, flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
