"""Generate golden input/output vectors by running the reference genome-kmers itself.

This script is test infrastructure.  It is run ONCE, in the build container, with the
reference checked out read-only at /root/reference; its outputs (``*.npz`` + ``manifest.json``
in this directory) are committed and travel to the GPU box, the script and the reference do not
need to.

How the reference is executed
-----------------------------
The reference (mrperkett/genome-kmers v1.0.1) is numpy + numba ``@jit``.  In this container
numba 0.54.1 is installed under /opt/conda but fails to import against the numpy that was later
installed next to it (``SystemError: initialization of _internal failed``) -- an ordinary
import error.  We therefore run the reference with numba's JIT replaced by the identity
decorator, which is what ``NUMBA_DISABLE_JIT=1`` does: the *same* Python source executes in the
interpreter.  The sort's third-party algorithm, ``numba.misc.quicksort`` (the reference's
``Kmers.sort`` calls ``quicksort.make_jit_quicksort``, kmers.py:1644), is loaded unmodified from
the installed numba package by file path; nothing of numba or of the reference is copied.

Run:  /opt/conda/bin/python3.9 tests/golden/make_golden.py
"""

import importlib.util
import json
import os
import sys
import tempfile
import textwrap
import time

import numpy as np

REF_SRC = "/root/reference/src"
NUMBA_QUICKSORT = "/opt/conda/lib/python3.9/site-packages/numba/misc/quicksort.py"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))


def build_numba_stub() -> str:
    """Write an identity-JIT numba package into a temp dir and return its path."""
    root = tempfile.mkdtemp(prefix="gk_numba_stub_")
    files = {
        "numba/__init__.py": """
            def jit(*args, **kwargs):
                if len(args) == 1 and callable(args[0]) and not kwargs:
                    return args[0]
                return lambda f: f
            njit = jit
        """,
        "numba/core/__init__.py": "",
        "numba/core/types.py": """
            import numpy as np
            uint8 = np.uint8
            unicode_type = str
            intp = int
        """,
        "numba/core/extending.py": """
            def register_jitable(f):
                return f
        """,
        "numba/typed/__init__.py": """
            class Dict(dict):
                @classmethod
                def empty(cls, key_type=None, value_type=None):
                    return cls()
        """,
        "numba/misc/__init__.py": "",
        # load numba's own pure-Python quicksort module from the installed package
        "numba/misc/quicksort.py": f"""
            import importlib.util as _u
            _spec = _u.spec_from_file_location("_numba_quicksort_src", {NUMBA_QUICKSORT!r})
            _mod = _u.module_from_spec(_spec)
            _spec.loader.exec_module(_mod)
            globals().update({{k: v for k, v in vars(_mod).items() if not k.startswith("__")}})
        """,
    }
    for rel, body in files.items():
        path = os.path.join(root, rel)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as fh:
            fh.write(textwrap.dedent(body))
    return root


sys.path.insert(0, REF_SRC)
sys.path.insert(0, build_numba_stub())

from numba.misc import quicksort  # noqa: E402  (stub -> numba's own quicksort.py)

from genome_kmers import kmers as gk  # noqa: E402
from genome_kmers.sequence_collection import SequenceCollection  # noqa: E402


# ---------------------------------------------------------------------------------------------
# inputs
# ---------------------------------------------------------------------------------------------


def random_seq(n: int, seed: int) -> str:
    """Same draw as genome_kmers.profiling.get_random_seq under np.random.seed(seed)."""
    np.random.seed(seed)
    bases = np.array(["A", "T", "G", "C"], dtype="U1")
    return "".join(np.random.choice(bases, n, replace=True))


def iupac_genome(seed: int) -> list:
    """Multi-contig genome with N runs, IUPAC letters and planted repeats (ties at k=31)."""
    rng = np.random.RandomState(seed)
    acgt = np.array(list("ACGT"))
    iupac = np.array(list("RYSWKMBDHVN"))
    repeat = "".join(rng.choice(acgt, 400))
    contigs = []
    for c, length in enumerate([3000, 1200, 5000, 64, 2500]):
        s = list("".join(rng.choice(acgt, length)))
        # planted copies of a shared repeat (exact) and a mutated copy
        if length > 1000:
            for _ in range(3):
                at = rng.randint(0, length - 400)
                s[at : at + 400] = list(repeat)
            at = rng.randint(0, length - 400)
            mutated = list(repeat)
            mutated[rng.randint(0, 400)] = "N"
            s[at : at + 400] = mutated
        # N runs at the ends and in the middle, sprinkled IUPAC codes
        if length > 1000:
            s[:50] = ["N"] * 50
            mid = length // 2
            s[mid : mid + 80] = ["N"] * 80
        for _ in range(max(1, length // 300)):
            s[rng.randint(0, length)] = rng.choice(iupac)
        contigs.append((f"ctg{c}", "".join(s)))
    return contigs


def repeat_genome(seed: int) -> list:
    """ACGT-only multi-contig genome with heavy exact repeats and homopolymers."""
    rng = np.random.RandomState(seed)
    acgt = np.array(list("ACGT"))
    unit = "".join(rng.choice(acgt, 97))
    contigs = []
    for c, length in enumerate([2000, 1500, 40, 3000]):
        s = list("".join(rng.choice(acgt, length)))
        if length >= 1500:
            for _ in range(6):
                at = rng.randint(0, length - 97)
                s[at : at + 97] = list(unit)
            at = rng.randint(0, length - 60)
            s[at : at + 60] = ["A"] * 60
        contigs.append((f"r{c}", "".join(s)))
    return contigs


# ---------------------------------------------------------------------------------------------
# reference calls
# ---------------------------------------------------------------------------------------------


def stable_sort(km: "gk.Kmers") -> np.ndarray:
    """The reference's own break_ties=True order (kmers.py:1654-1731) through numba quicksort."""
    lt = km.get_is_less_than_func(validate_kmers=True, break_ties=True)
    qs = quicksort.make_jit_quicksort(lt=lt, is_argsort=False)
    arr = km.kmer_sba_start_indices.copy()
    qs.run_quicksort(arr)
    return arr


FILTER_SPECS = {
    "keep_all": lambda p: gk.kmer_filter_keep_all,
    "length": lambda p: gk.gen_kmer_length_filter_func(p["min_kmer_len"]),
    "homopolymer": lambda p: gk.gen_kmer_homopolymer_filter_func(p["max_homopolymer_size"], p["kmer_len"]),
    "gc": lambda p: gk.gen_kmer_gc_content_filter_func(p["min_gc"], p["max_gc"], p["kmer_len"]),
    "no_ambiguous": lambda p: gk.gen_no_ambiguous_bases_filter(p["kmer_len"]),
    "crispr_ngg": lambda p: gk.crispr_ngg_pam_filter,
}


def run_query(km, q):
    """Run one counting/grouping query on a sorted Kmers object; capture result or error."""
    filt = FILTER_SPECS[q["filter"]["kind"]](q["filter"])
    try:
        if q["op"] == "group_counts":
            hist, total = km.get_kmer_group_counts(
                q["kmer_len"], filt, q["min_group_size"], q["max_group_size"], q["max_counts_bin"]
            )
            return {"hist": hist.tolist(), "total": int(total)}
        if q["op"] == "count":
            total = km.get_kmer_count(q["kmer_len"], filt, q["min_group_size"], q["max_group_size"])
            return {"total": int(total)}
        if q["op"] == "get_kmers":
            out = []
            for t in km.get_kmers(
                q["kmer_len"],
                kmer_filter_func=filt,
                kmer_info_to_yield=q.get("info", "minimum"),
                min_group_size=q["min_group_size"],
                max_group_size=q["max_group_size"],
                yield_first_n=q.get("yield_first_n"),
                one_based_seq_index=q.get("one_based", False),
            ):
                out.append([int(x) if isinstance(x, (int, np.integer)) else x for x in t])
            return {"kmers": out}
        raise ValueError(q["op"])
    except (ValueError, AssertionError) as e:  # reference raises these from filters / guards
        return {"error": type(e).__name__, "message": str(e)}


def make_case(name, seq_list, min_k, max_k, queries, store_unsorted=True):
    t0 = time.time()
    sc = SequenceCollection(sequence_list=seq_list, strands_to_load="forward")
    km = gk.Kmers(sc, min_kmer_len=min_k, max_kmer_len=max_k)
    unsorted = km.kmer_sba_start_indices.copy()
    stable = stable_sort(km)
    km.sort()
    default = km.kmer_sba_start_indices.copy()

    # queries on the reference's default tie order, and on the stable order
    res_default = [run_query(km, q) for q in queries]
    km.kmer_sba_start_indices = stable.copy()
    res_stable = [run_query(km, q) for q in queries]
    km.kmer_sba_start_indices = default

    arrays = {
        "sba": sc.forward_sba,
        "seg_starts": sc._forward_sba_seg_starts,
        "starts_default": default,
        "starts_stable": stable,
    }
    if store_unsorted:
        arrays["starts_unsorted"] = unsorted
    np.savez_compressed(os.path.join(OUT_DIR, f"{name}.npz"), **arrays)
    entry = {
        "name": name,
        "record_names": [r for r, _ in seq_list],
        "min_kmer_len": min_k,
        "max_kmer_len": max_k,
        "num_kmers": int(len(default)),
        "ties_differ": bool((default != stable).any()),
        "queries": queries,
        "results_default_order": res_default,
        "results_stable_order": res_stable,
        "seconds": round(time.time() - t0, 2),
    }
    print(f"{name}: n={len(default)} ties_differ={entry['ties_differ']} {entry['seconds']}s", flush=True)
    return entry


def q(op, kmer_len, filt=None, ming=1, maxg=None, bins=16, **kw):
    d = {
        "op": op,
        "kmer_len": kmer_len,
        "filter": filt or {"kind": "keep_all"},
        "min_group_size": ming,
        "max_group_size": maxg,
        "max_counts_bin": bins,
    }
    d.update(kw)
    return d


SEQ_LIST_2 = [("chr1", "ATCGAATTAG"), ("chr2", "GGATCTTGCATT"), ("chr3", "GTGATTGACCCCT")]


def main():
    only = set(sys.argv[1:])
    manifest_path = os.path.join(OUT_DIR, "manifest.json")
    manifest = {}
    if os.path.exists(manifest_path):
        with open(manifest_path) as fh:
            manifest = {c["name"]: c for c in json.load(fh)["cases"]}

    cases = []

    # docs example (docs/overview.rst), every (min, max) combination incl. max=None
    for mn in range(1, 10):
        for mx in list(range(mn, 10)) + [None]:
            qs = [
                q("group_counts", 1, bins=15),
                q("group_counts", mn, bins=6),
                q("count", mn, ming=2),
                q("get_kmers", mn, yield_first_n=None),
                q("get_kmers", mn, ming=2, yield_first_n=1),
            ]
            cases.append((f"seq2_min{mn}_max{mx if mx is not None else 'None'}", SEQ_LIST_2, mn, mx, qs))

    # C1: 10 kb random ACGT, seed 42, k=5 (BASELINE config 0)
    c1_queries = [
        q("group_counts", 5, bins=64),
        q("group_counts", 5, ming=3, maxg=12, bins=64),
        q("group_counts", 3, bins=256),
        q("count", 5, maxg=1),
        q("count", 5, filt={"kind": "homopolymer", "max_homopolymer_size": 2, "kmer_len": 5}),
        q("count", 5, filt={"kind": "gc", "min_gc": 0.4, "max_gc": 0.6, "kmer_len": 5}),
        q("get_kmers", 5, ming=20, yield_first_n=2),
    ]
    cases.append(("c1_seed42_10kb_k5", [("chr0", random_seq(10_000, 42))], 5, 5, c1_queries))

    # random single contig k=31 (no ties expected), and a bounded variable-length case
    r31 = [("chr0", random_seq(10_000, 7))]
    cases.append(("rand10k_k31", r31, 31, 31, [q("group_counts", 31, bins=8), q("group_counts", 12, bins=32)]))

    # IUPAC / N / multi-contig / planted repeats at k=31
    ig = iupac_genome(11)
    iq = [
        q("group_counts", 31, bins=32),
        q("group_counts", 31, ming=2, bins=32),
        q("group_counts", 20, bins=32),
        q("count", 31, filt={"kind": "no_ambiguous", "kmer_len": 31}),
        q("count", 31, filt={"kind": "homopolymer", "max_homopolymer_size": 4, "kmer_len": 31}),
        q("count", 31, filt={"kind": "gc", "min_gc": 0.3, "max_gc": 0.55, "kmer_len": 31}),
        q("count", 31, filt={"kind": "length", "min_kmer_len": 31}),
        q("get_kmers", 31, ming=3, yield_first_n=1, info="full"),
        q("get_kmers", 31, ming=3, yield_first_n=2, info="full", one_based=True),
    ]
    cases.append(("iupac_k31", ig, 31, 31, iq))

    # ACGT-only with heavy repeats: fixed k=31, bounded variable length, and suffix mode
    rg = repeat_genome(5)
    rq = [
        q("group_counts", 31, bins=64),
        q("group_counts", 8, bins=64),
        q("count", 31, ming=2, maxg=5),
        q("count", 23, filt={"kind": "crispr_ngg"}),
        q("count", 31, filt={"kind": "homopolymer", "max_homopolymer_size": 3, "kmer_len": 31}),
        q("get_kmers", 31, ming=4, yield_first_n=3),
    ]
    cases.append(("repeat_k31", rg, 31, 31, rq))
    cases.append(("repeat_k40", rg, 40, 40, [q("group_counts", 40, bins=64)]))
    cases.append(("repeat_min10_max40", rg, 10, 40, [q("group_counts", 10, bins=64), q("count", 40, ming=2)]))
    small_rg = [(n, s[:300]) for n, s in rg if len(s) >= 300] + [("tail", rg[2][1])]
    cases.append(
        ("repeat_suffix_min4", small_rg, 4, None, [q("group_counts", 4, bins=64), q("group_counts", None, bins=8)])
    )
    ig_small = [(n, s[:400]) for n, s in ig if len(s) >= 400]
    cases.append(("iupac_min6_max25", ig_small, 6, 25, [q("group_counts", 6, bins=64), q("count", 25, ming=2)]))
    cases.append(("iupac_suffix_min2", ig_small, 2, None, [q("group_counts", 2, bins=64), q("count", 9, ming=2)]))

    # filters that raise (the reference's error sites), on the docs example
    eq = [
        q("count", 3, filt={"kind": "homopolymer", "max_homopolymer_size": 2, "kmer_len": 12}),
        q("count", 3, filt={"kind": "gc", "min_gc": 0.0, "max_gc": 1.0, "kmer_len": 11}),
        q("count", 3, filt={"kind": "no_ambiguous", "kmer_len": 11}),
        q("count", 3, filt={"kind": "no_ambiguous", "kmer_len": 40}),
        q("count", 3, filt={"kind": "crispr_ngg"}),
        q("count", 3, filt={"kind": "homopolymer", "max_homopolymer_size": 1, "kmer_len": 3}),
        q("count", 3, filt={"kind": "length", "min_kmer_len": 9}),
    ]
    cases.append(("seq2_filter_errors", SEQ_LIST_2, 3, 3, eq))

    for name, seq_list, mn, mx, qs in cases:
        if only and name not in only:
            continue
        manifest[name] = make_case(name, seq_list, mn, mx, qs)

    with open(manifest_path, "w") as fh:
        json.dump({"generator": "tests/golden/make_golden.py", "reference": "mrperkett/genome-kmers v1.0.1",
                   "cases": list(manifest.values())}, fh, indent=1)


if __name__ == "__main__":
    main()
