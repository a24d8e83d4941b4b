"""CPU parity oracle for the genome-kmers hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this
module, and only as the checker / the timed reference algorithm.  The product (genome_kmers,
libgkm.so) never imports, links or calls it.

It wraps ``gk_oracle.c`` (a C restatement of the reference's enumerate / comparator / numba
quicksort / filters / group generator, each function citing the reference file:line it follows)
and adds a numpy restatement of the key encoding the device emits.

Pinning: every function is checked against the golden vectors in ``tests/golden/`` that were
produced by running the reference itself (``tests/golden/make_golden.py``).
"""

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "libgk_oracle.so"
DOLLAR = 36

_lib = None

_U8P = ctypes.POINTER(ctypes.c_uint8)
_U32P = ctypes.POINTER(ctypes.c_uint32)
_I64P = ctypes.POINTER(ctypes.c_int64)
_U64P = ctypes.POINTER(ctypes.c_uint64)

FILTER_KINDS = {"keep_all": 0, "length": 1, "homopolymer": 2, "gc": 3, "no_ambiguous": 4, "crispr_ngg": 5}

ERRORS = {
    -1: "no_bases", -2: "too_short", -3: "stack", -10: "homo_len", -11: "gc_len", -12: "gc_oob",
    -13: "ambig_len", -14: "ambig_seg", -15: "crispr_len",
}


def build():
    """Compile gk_oracle.c with gcc (idempotent)."""
    src = HERE / "gk_oracle.c"
    if LIB.exists() and LIB.stat().st_mtime >= src.stat().st_mtime:
        return LIB
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(str(LIB))
        L.gko_compare.argtypes = [_U8P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64, _I64P]
        L.gko_compare.restype = ctypes.c_int
        L.gko_kmer_count.argtypes = [_U32P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64]
        L.gko_kmer_count.restype = ctypes.c_int64
        L.gko_enumerate.argtypes = [_U32P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64, _U32P]
        L.gko_enumerate.restype = None
        L.gko_quicksort.argtypes = [_U8P, ctypes.c_uint64, _U32P, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_int, ctypes.c_int, _U64P]
        L.gko_quicksort.restype = ctypes.c_int
        L.gko_filter.argtypes = [_U8P, ctypes.c_uint64, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                 ctypes.c_uint64]
        L.gko_filter.restype = ctypes.c_int
        L.gko_group_scan.argtypes = [_U8P, ctypes.c_uint64, _U32P, ctypes.c_uint64, ctypes.c_int, ctypes.c_int64,
                                     ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                     ctypes.c_int64, ctypes.c_int64, _I64P, ctypes.c_int64, _I64P, _I64P, _I64P,
                                     _I64P, ctypes.c_int64, _I64P, _U64P]
        L.gko_group_scan.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


class OracleError(Exception):
    def __init__(self, code, idx):
        super().__init__(f"{ERRORS.get(code, code)} at sba index {idx}")
        self.kind = ERRORS.get(code, str(code))
        self.idx = idx


# ---------------------------------------------------------------------------------------------
def compare(sba, a, b, max_kmer_len=None):
    """compare_sba_kmers_lexicographically (kmers.py:306-397) -> (cmp, last)."""
    sba = np.ascontiguousarray(sba, dtype=np.uint8)
    last = ctypes.c_int64(0)
    r = lib().gko_compare(_p(sba, ctypes.c_uint8), sba.size, a, b, -1 if max_kmer_len is None else max_kmer_len,
                          ctypes.byref(last))
    if r == 2:
        raise AssertionError("There were no valid kmer bases to compare")
    return r, last.value


def enumerate_starts(sba, seg_starts, min_kmer_len):
    """Kmers._initialize_single_pass (kmers.py:789-861)."""
    seg = np.ascontiguousarray(seg_starts, dtype=np.uint32)
    n = lib().gko_kmer_count(_p(seg, ctypes.c_uint32), seg.size, len(sba), min_kmer_len)
    out = np.empty(n, dtype=np.uint32)
    lib().gko_enumerate(_p(seg, ctypes.c_uint32), seg.size, len(sba), min_kmer_len, _p(out, ctypes.c_uint32))
    return out


def quicksort(sba, starts, min_kmer_len, max_kmer_len=None, break_ties=False, validate=True):
    """Kmers.sort through numba's quicksort (kmers.py:1624-1731); returns a sorted copy."""
    sba = np.ascontiguousarray(sba, dtype=np.uint8)
    arr = np.array(starts, dtype=np.uint32, copy=True)
    err = ctypes.c_uint64(0)
    rc = lib().gko_quicksort(_p(sba, ctypes.c_uint8), sba.size, _p(arr, ctypes.c_uint32), arr.size, min_kmer_len,
                             -1 if max_kmer_len is None else max_kmer_len, int(break_ties), int(validate),
                             ctypes.byref(err))
    if rc:
        raise OracleError(rc, err.value)
    return arr


def filter_params(spec: dict):
    """(kind, p0, p1, p2) of a golden filter spec (same parameter derivation as kmers.py:142-144)."""
    k = spec["kind"]
    if k == "length":
        return 1, spec["min_kmer_len"], 0, 0
    if k == "homopolymer":
        return 2, spec["max_homopolymer_size"], spec["kmer_len"], 0
    if k == "gc":
        kl = spec["kmer_len"]
        return 3, int(np.ceil(kl * spec["min_gc"])), int(np.floor(kl * spec["max_gc"])), kl
    if k == "no_ambiguous":
        return 4, spec["kmer_len"], 0, 0
    if k == "crispr_ngg":
        return 5, 0, 0, 0
    return 0, 0, 0, 0


def group_scan(sba, starts, kmer_len, filt=(0, 0, 0, 0), min_group_size=1, max_group_size=None,
               yield_first_n=None, max_counts_bin=None, is_sorted=True):
    """kmer_info_by_group_generator (+ get_kmer_group_size_hist when max_counts_bin is given).

    Returns (hist, total) in histogram mode, else a list of (kmer_num, yielded, total).
    """
    sba = np.ascontiguousarray(sba, dtype=np.uint8)
    st = np.ascontiguousarray(starts, dtype=np.uint32)
    kind, p0, p1, p2 = filt
    err = ctypes.c_uint64(0)
    total = ctypes.c_int64(0)
    ycount = ctypes.c_int64(0)
    null = ctypes.POINTER(ctypes.c_int64)()
    common = (_p(sba, ctypes.c_uint8), sba.size, _p(st, ctypes.c_uint32), st.size, int(is_sorted),
              -1 if kmer_len is None else kmer_len, kind, p0, p1, p2, min_group_size,
              -1 if max_group_size is None else max_group_size)
    if max_counts_bin is not None:
        hist = np.zeros(max_counts_bin + 1, dtype=np.int64)
        rc = lib().gko_group_scan(*common, 1, _p(hist, ctypes.c_int64), max_counts_bin, ctypes.byref(total), null,
                                  null, null, 0, ctypes.byref(ycount), ctypes.byref(err))
        if rc:
            raise OracleError(rc, err.value)
        return hist, total.value
    cap = st.size
    num = np.zeros(cap, dtype=np.int64)
    y = np.zeros(cap, dtype=np.int64)
    t = np.zeros(cap, dtype=np.int64)
    rc = lib().gko_group_scan(*common, -1 if yield_first_n is None else yield_first_n, null, 0, ctypes.byref(total),
                              _p(num, ctypes.c_int64), _p(y, ctypes.c_int64), _p(t, ctypes.c_int64), cap,
                              ctypes.byref(ycount), ctypes.byref(err))
    if rc:
        raise OracleError(rc, err.value)
    m = ycount.value
    return list(zip(num[:m].tolist(), y[:m].tolist(), t[:m].tolist()))


# ---------------------------------------------------------------------------------------------
# key encoding -- numpy restatement used to check the device keys
# ---------------------------------------------------------------------------------------------
CODE4_ORDER = b"ABCDGHKMNRSTVWY"
CODE4 = np.zeros(256, dtype=np.uint64)
for _i, _c in enumerate(CODE4_ORDER):
    CODE4[_c] = _i + 1
CODE2 = np.zeros(256, dtype=np.uint64)
for _i, _c in enumerate(b"ACGT"):
    CODE2[_c] = _i


def key_spec(is_acgt: bool, min_kmer_len: int, max_kmer_len: int):
    """(bits, symbols, lenbits, words) of the direct key for a bounded sort length."""
    bits = 2 if is_acgt else 4
    lenbits = int(max_kmer_len).bit_length() if (bits == 2 and max_kmer_len != min_kmer_len) else 0
    total = bits * max_kmer_len + lenbits
    return bits, max_kmer_len, lenbits, (total + 63) // 64


def encode_keys(sba, starts, bits, symbols, lenbits, words):
    """Keys of the k-mers at starts, shape (n, words), word 0 most significant."""
    sba = np.asarray(sba, dtype=np.uint8)
    starts = np.asarray(starts, dtype=np.int64)
    n = starts.size
    padded = np.concatenate([sba, np.full(symbols + 1, DOLLAR, dtype=np.uint8)])
    win = padded[starts[:, None] + np.arange(symbols)[None, :]]
    term = np.cumsum(win == DOLLAR, axis=1) > 0
    length = np.where(term.any(axis=1), term.argmax(axis=1), symbols).astype(np.uint64)
    codes = (CODE2 if bits == 2 else CODE4)[win]
    codes[term] = 0
    lsw = np.zeros((n, words), dtype=np.uint64)  # least significant word first
    for t in range(symbols):
        off = lenbits + bits * (symbols - 1 - t)
        w, sh = divmod(off, 64)
        lsw[:, w] |= codes[:, t] << np.uint64(sh)
        if sh + bits > 64:
            lsw[:, w + 1] |= codes[:, t] >> np.uint64(64 - sh)
    if lenbits:
        lsw[:, 0] |= length
    return lsw[:, ::-1].copy()


# ---------------------------------------------------------------------------------------------
# canonical k-mers (C5) -- this build's extension: the reference defines no canonical k-mer
# (kmers.py:689-696), so the ORDER below is parity-unpinned by the reference; the complement
# mapping it uses is the reference's and is pinned by tests/golden/complement.npz.
# ---------------------------------------------------------------------------------------------
# SequenceCollection._get_complement_mapping_array (sequence_collection.py:402-433)
COMPLEMENT_LUT = np.zeros(256, dtype=np.uint8)
for _a, _b in zip(b"ACGTRYSWKMBDHVN$", b"TGCAYRSWMKVHDBN$"):
    COMPLEMENT_LUT[_a] = _b


def reverse_complement(sba):
    """reverse_complement_sba(sba, lut) with inplace=False (sequence_collection.py:42-73)."""
    return COMPLEMENT_LUT[np.asarray(sba, dtype=np.uint8)[::-1]]


def canonical_windows(sba, starts, k):
    """(canonical k-mer bytes (n, k), is_rc (n,)) of the fixed-length k-mers at starts: the
    smaller of the k-mer and its reverse complement under the reference's byte order
    (compare_sba_kmers_lexicographically, kmers.py:306-397; equal lengths, no '$' inside)."""
    sba = np.asarray(sba, dtype=np.uint8)
    starts = np.asarray(starts, dtype=np.int64)
    win = sba[starts[:, None] + np.arange(k)[None, :]]
    rc = COMPLEMENT_LUT[win[:, ::-1]]
    diff = win != rc
    first = diff.argmax(axis=1)
    rows = np.arange(len(starts))
    is_rc = diff.any(axis=1) & (rc[rows, first] < win[rows, first])
    return np.where(is_rc[:, None], rc, win), is_rc


def canonical_sort(sba, starts, k):
    """Starts ordered by canonical k-mer, equal canonical k-mers by ascending start (the device's
    break_ties order)."""
    starts = np.asarray(starts, dtype=np.uint32)
    canon, _ = canonical_windows(sba, starts, k)
    order = np.lexsort([starts] + [canon[:, j] for j in range(k - 1, -1, -1)])
    return starts[order]


def canonical_group_hist(sba, sorted_starts, k, max_counts_bin=1000000):
    """Group-size histogram + total of equal canonical k-mers over a canonical-sorted array, with
    get_kmer_group_size_hist's binning (kmers.py:454-520: overflow into the last bin)."""
    hist = np.zeros(max_counts_bin + 1, dtype=np.int64)
    if len(sorted_starts) == 0:
        return hist, 0
    canon, _ = canonical_windows(sba, sorted_starts, k)
    heads = np.concatenate([[True], (canon[1:] != canon[:-1]).any(axis=1)])
    gs = np.flatnonzero(heads)
    sizes = np.diff(np.append(gs, len(sorted_starts)))
    np.add.at(hist, np.minimum(sizes, max_counts_bin), 1)
    return hist, int(sizes.sum())


def canonical_keys(sba, starts, k, bits):
    """Encoded canonical keys (n, words), word 0 most significant (DESIGN.md §2 encoding of the
    canonical bytes)."""
    canon, _ = canonical_windows(sba, starts, k)
    flat = np.concatenate([canon, np.full((len(canon), 1), DOLLAR, dtype=np.uint8)], axis=1).ravel()
    rows = np.arange(len(canon), dtype=np.int64) * (k + 1)
    words = (bits * k + 63) // 64
    return encode_keys(flat, rows, bits, k, 0, words)
