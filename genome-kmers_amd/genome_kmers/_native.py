"""ctypes binding of libgkm.so (include/gkm.h) -- the only way this package reaches the GPU.

There is no CPU fallback: if the library is missing or no HIP device is visible, every call that
needs the engine raises.  ``Engine`` owns one ``gk_ctx`` (one device, one stream, device buffers).
"""

import ctypes
import os
from pathlib import Path

import numpy as np

GK_OK = 0
GK_E_ARG = -1
GK_E_HIP = -2
GK_E_OOM = -3
GK_E_UNSUPPORTED = -4
GK_E_ALPHABET = -5
GK_E_STATE = -6
GK_E_FILTER = -7
GK_E_LIMIT = -8
GK_E_NO_BASES = -9
GK_E_IO = -10
GK_E_FASTA_NAME = -11
GK_E_FASTA_LAYOUT = -12

# gk_filter_kind
FILTER_KEEP_ALL = 0
FILTER_LENGTH = 1
FILTER_HOMOPOLYMER = 2
FILTER_GC = 3
FILTER_NO_AMBIGUOUS = 4
FILTER_CRISPR_NGG = 5
FILTER_MASK = 6

# gk_filter_error
FERR_HOMO_LEN = 1
FERR_GC_LEN = 2
FERR_GC_OOB = 3
FERR_AMBIG_LEN = 4
FERR_AMBIG_SEG = 5
FERR_CRISPR_LEN = 6

LIB_PATH = Path(__file__).with_name("libgkm.so")
# tuning only: GKM_LIB names another build of the same library (A/B of compile-time variants)
if os.environ.get("GKM_LIB"):
    LIB_PATH = Path(os.environ["GKM_LIB"]).resolve()

# every symbol include/gkm.h declares (checked by tests/test_native_abi.py)
EXPORTED = (
    "gk_create", "gk_destroy", "gk_last_error", "gk_sync", "gk_device_count", "gk_set_sequence",
    "gk_alphabet_is_acgt", "gk_enumerate", "gk_set_start_indices", "gk_sort", "gk_num_kmers",
    "gk_copy_start_indices", "gk_copy_start_range", "gk_key_layout", "gk_copy_keys", "gk_set_filter_mask",
    "gk_set_group_heads", "gk_group_hist", "gk_group_members", "gk_unique_counts", "gk_copy_unique", "gk_device_unique", "gk_device_views",
    "gk_profile_enable", "gk_profile_report", "gk_stream", "gk_shard_bucket_bits", "gk_shard_partition",
    "gk_shard_sort", "gk_fasta_open", "gk_fasta_fill", "gk_fasta_close", "gk_locate", "gk_copy_strands",
    "gk_shard_histogram", "gk_shard_sort_range", "gk_shard_class_b", "gk_shard_class_b_copy",
    "gk_shard_sort_range_b", "gk_rank_mode", "gk_reference_random_bases",
    "gk_copy_sequence", "gk_sort_hint", "gk_resident_packed", "gk_set_option",
)

SORT_CANONICAL = 1  # GK_SORT_CANONICAL
SORT_QUICKSORT_ORDER = 2  # GK_SORT_QUICKSORT_ORDER
SHARD_STARTS_ONLY = 4  # GK_SHARD_STARTS_ONLY


class GkFilter(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("pad", ctypes.c_int32), ("p0", ctypes.c_int64),
                ("p1", ctypes.c_int64), ("p2", ctypes.c_int64)]


class GkError(RuntimeError):
    """A libgkm call failed; ``code`` is the gk_status."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"libgkm error {code}: {msg}")
        self.code = code
        self.msg = msg


class FilterRaised(GkError):
    """A built-in filter raised on the device; carries the reference's error site."""

    def __init__(self, ferr: int, sba_idx: int):
        super().__init__(GK_E_FILTER, f"filter error {ferr} at sba index {sba_idx}")
        self.ferr = ferr
        self.sba_idx = sba_idx


_lib = None

_P = ctypes.c_void_p
_U32P = ctypes.POINTER(ctypes.c_uint32)
_U64P = ctypes.POINTER(ctypes.c_uint64)
_I64P = ctypes.POINTER(ctypes.c_int64)
_I32P = ctypes.POINTER(ctypes.c_int32)
_U8P = ctypes.POINTER(ctypes.c_uint8)

_SIGS = {
    "gk_create": ([ctypes.POINTER(_P), ctypes.c_int], ctypes.c_int),
    "gk_destroy": ([_P], None),
    "gk_last_error": ([_P], ctypes.c_char_p),
    "gk_sync": ([_P], ctypes.c_int),
    "gk_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "gk_set_sequence": ([_P, _U8P, ctypes.c_uint64, _U32P, ctypes.c_uint64], ctypes.c_int),
    "gk_sort_hint": ([_P, ctypes.c_uint32, ctypes.c_uint32], ctypes.c_int),
    "gk_alphabet_is_acgt": ([_P, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "gk_enumerate": ([_P, ctypes.c_uint32, _U64P], ctypes.c_int),
    "gk_set_start_indices": ([_P, _U32P, ctypes.c_uint64, ctypes.c_uint32], ctypes.c_int),
    "gk_sort": ([_P, ctypes.c_uint32, ctypes.c_uint32], ctypes.c_int),
    "gk_num_kmers": ([_P, _U64P], ctypes.c_int),
    "gk_copy_start_indices": ([_P, _U32P, ctypes.c_uint64], ctypes.c_int),
    "gk_copy_start_range": ([_P, ctypes.c_uint64, _U32P, ctypes.c_uint64], ctypes.c_int),
    "gk_key_layout": ([_P, _U32P, _U32P, _U32P], ctypes.c_int),
    "gk_copy_keys": ([_P, _U64P, ctypes.c_uint64], ctypes.c_int),
    "gk_set_filter_mask": ([_P, _U8P, ctypes.c_uint64], ctypes.c_int),
    "gk_set_group_heads": ([_P, _U8P, ctypes.c_uint64], ctypes.c_int),
    "gk_group_hist": ([_P, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(GkFilter), ctypes.c_int64, ctypes.c_int64,
                       ctypes.c_int64, _I64P, _I64P, _I32P, _U64P], ctypes.c_int),
    "gk_group_members": ([_P, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(GkFilter), ctypes.c_int64,
                          ctypes.c_int64, ctypes.c_int64, _U64P, _U32P, _U32P, ctypes.c_uint64, _U64P, _I32P,
                          _U64P], ctypes.c_int),
    "gk_unique_counts": ([_P, _U64P], ctypes.c_int),
    "gk_copy_unique": ([_P, _U64P, _U32P, ctypes.c_uint64], ctypes.c_int),
    "gk_device_unique": ([_P, ctypes.POINTER(_P), ctypes.POINTER(_P), _U64P], ctypes.c_int),
    "gk_device_views": ([_P, ctypes.POINTER(_P), ctypes.POINTER(_P), _U64P, _U32P], ctypes.c_int),
    "gk_profile_enable": ([_P, ctypes.c_int], ctypes.c_int),
    "gk_profile_report": ([_P, ctypes.c_char_p, ctypes.c_uint64], ctypes.c_int),
    "gk_stream": ([_P, ctypes.POINTER(_P)], ctypes.c_int),
    "gk_shard_bucket_bits": ([], ctypes.c_int),
    "gk_shard_partition": ([_P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _P, _P,
                            ctypes.c_uint64, _U64P, _U64P], ctypes.c_int),
    "gk_shard_sort": ([_P, _P, _P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _U64P, _U64P, _U32P,
                       ctypes.c_uint32], ctypes.c_int),
    "gk_shard_histogram": ([_P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _U64P, _U32P],
                           ctypes.c_int),
    "gk_shard_sort_range": ([_P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _U64P],
                            ctypes.c_int),
    "gk_shard_class_b": ([_P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _U64P, _U64P,
                          _U64P], ctypes.c_int),
    "gk_shard_class_b_copy": ([_P, _U32P, ctypes.c_uint64, _U32P, ctypes.c_uint64], ctypes.c_int),
    "gk_shard_sort_range_b": ([_P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _U32P,
                               ctypes.c_uint64, _U32P, ctypes.c_uint64, _U64P], ctypes.c_int),
    "gk_fasta_open": ([ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(_P), _U64P, _U64P, _U64P], ctypes.c_int),
    "gk_fasta_fill": ([_P, _U8P, ctypes.c_uint64, _U32P, ctypes.c_char_p, _U8P], ctypes.c_int),
    "gk_fasta_close": ([_P], None),
    "gk_locate": ([_P, _U64P, ctypes.c_uint64, _U32P, _U32P], ctypes.c_int),
    "gk_copy_strands": ([_P, _U8P, ctypes.c_uint64], ctypes.c_int),
    "gk_rank_mode": ([_P, ctypes.c_int, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "gk_reference_random_bases": ([_U8P, ctypes.c_uint64, ctypes.c_uint32], ctypes.c_int),
    "gk_copy_sequence": ([_P, _U8P, ctypes.c_uint64], ctypes.c_int),
    "gk_resident_packed": ([_P, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "gk_set_option": ([ctypes.c_char_p, ctypes.c_char_p], ctypes.c_int),
}


def _share_hip_runtime():
    """One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64 (soname
    libamdhip64.so.7, loaded by torch as "libamdhip64.so"); libgkm needs libamdhip64.so.7.  If
    libgkm loaded /opt/rocm's copy first, torch would later load a second runtime and fail to see
    the GPU ("No HIP GPUs are available").  Loading torch's copy first (global, without importing
    torch) makes both bind the same runtime, whichever is imported first."""
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    for root in spec.submodule_search_locations:
        hip = Path(root) / "lib" / "libamdhip64.so"
        if hip.exists():
            ctypes.CDLL(str(hip), mode=ctypes.RTLD_GLOBAL)
            return


GROUPS_FROM_HEADS = 2  # gk_group_hist / gk_group_members: groups from gk_set_group_heads


def _group_mode(is_sorted) -> int:
    return GROUPS_FROM_HEADS if is_sorted == GROUPS_FROM_HEADS else int(bool(is_sorted))


def load_library(path: Path = LIB_PATH) -> ctypes.CDLL:
    """Load libgkm.so (raises if it has not been built -- there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not path.exists():
        raise RuntimeError(
            f"libgkm.so not found at {path}; build it with `make -C genome-kmers_amd/csrc` "
            "(genome_kmers has no CPU fallback)"
        )
    _share_hip_runtime()
    lib = ctypes.CDLL(str(path))
    for name, (args, res) in _SIGS.items():
        if os.environ.get("GKM_LIB") and not hasattr(lib, name):
            continue  # an older build under A/B (tuning only): entry points it lacks stay unbound
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


class FastaLayoutError(Exception):
    """gk_fasta_fill found bytes that would not fill the sba exactly (the reference asserts)."""


def read_fasta(path, n_threads: int = 0):
    """FASTA -> (sba uint8, seg_starts uint32, names list[str], bad byte values) with libgkm's
    multithreaded host parser (gk_fasta_open / gk_fasta_fill); the caller applies the reference's
    checks.  The sba length is total_seq_len + num_records - 1, allocated exactly as
    sequence_collection.py:531-533 does (so an empty file fails the same way)."""
    lib = load_library()
    with open(path, "rb"):  # the reference's open(): FileNotFoundError etc. with its messages
        pass
    h = _P()
    nrec, total, nbytes = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    rc = lib.gk_fasta_open(str(path).encode(), int(n_threads), ctypes.byref(h), ctypes.byref(nrec),
                           ctypes.byref(total), ctypes.byref(nbytes))
    if rc != GK_OK:
        raise OSError(f"cannot map {path} (libgkm error {rc})")
    try:
        sba_len = int(total.value) + int(nrec.value) - 1
        sba = np.zeros(sba_len, dtype=np.uint8)
        seg_starts = np.zeros(int(nrec.value), dtype=np.uint32)
        names = ctypes.create_string_buffer(max(int(nbytes.value), 1))
        bad = np.zeros(256, dtype=np.uint8)
        rc = lib.gk_fasta_fill(h, _ptr(sba, ctypes.c_uint8), sba_len, _ptr(seg_starts, ctypes.c_uint32), names,
                               _ptr(bad, ctypes.c_uint8))
    finally:
        lib.gk_fasta_close(h)
    if rc == GK_E_FASTA_NAME:
        raise IndexError("list index out of range")  # line[1:].strip().split()[0] on an empty name
    if rc == GK_E_FASTA_LAYOUT:
        raise FastaLayoutError()
    if rc != GK_OK:
        raise GkError(rc, "gk_fasta_fill failed")
    raw = names.raw[: int(nbytes.value)]
    name_list = [b.decode("utf-8") for b in raw.split(b"\0")[:-1]] if nrec.value else []
    return sba, seg_starts, name_list, set(np.flatnonzero(bad).tolist())


def reference_random_bases(n: int, seed: int) -> np.ndarray:
    """The reference's profiling genome (profiling.get_random_seq after np.random.seed(seed)) as n
    ASCII bytes, from libgkm's host MT19937 (gk_reference_random_bases)."""
    out = np.empty(n, dtype=np.uint8)
    lib = load_library()
    if os.environ.get("GKM_LIB") and not hasattr(lib, "gk_reference_random_bases"):
        # an older build under A/B (tuning only): the in-tree library's generator
        lib = ctypes.CDLL(str(Path(__file__).with_name("libgkm.so")))
        lib.gk_reference_random_bases.argtypes = _SIGS["gk_reference_random_bases"][0]
    rc = lib.gk_reference_random_bases(_ptr(out, ctypes.c_uint8), n, int(seed) & 0xFFFFFFFF)
    if rc != GK_OK:
        raise GkError(rc, "gk_reference_random_bases failed")
    return out


class _Options(dict):
    """libgkm's test and tuning overrides (gk_set_option), as a dict: ``options["GKM_X"] = "1"`` sets
    one, ``del options["GKM_X"]`` clears it -- so pytest's ``monkeypatch.setitem(options, ...)``
    restores the library state after a test.  Process-wide; names start with GKM_."""

    def __setitem__(self, name, value):
        rc = load_library().gk_set_option(name.encode(), str(value).encode())
        if rc != GK_OK:
            raise GkError(rc, f"gk_set_option({name!r}) failed")
        super().__setitem__(name, str(value))

    def __delitem__(self, name):
        super().__delitem__(name)  # (KeyError if unset, as a dict)
        load_library().gk_set_option(name.encode(), None)


options = _Options()


def _ptr(arr: np.ndarray, ctype):
    return arr.ctypes.data_as(ctypes.POINTER(ctype))


def device_count() -> int:
    lib = load_library()
    n = ctypes.c_int(0)
    if lib.gk_device_count(ctypes.byref(n)) != GK_OK:
        return 0
    return n.value


def default_device() -> int:
    return int(os.environ.get("GENOME_KMERS_DEVICE", os.environ.get("LOCAL_RANK", "0")))


class Engine:
    """One libgkm context: a sequence byte array resident in HBM plus its k-mer arrays."""

    def __init__(self, device: int = None):
        self.lib = load_library()
        self.device = default_device() if device is None else device
        self.ctx = _P()
        rc = self.lib.gk_create(ctypes.byref(self.ctx), self.device)
        if rc != GK_OK:
            self.ctx = None
            raise GkError(rc, f"cannot create a HIP context on device {self.device}: genome_kmers needs an "
                              "MI355X (gfx950) GPU and has no CPU fallback")
        self.n = 0

    def __del__(self):
        ctx = getattr(self, "ctx", None)
        if ctx:
            self.lib.gk_destroy(ctx)
            self.ctx = None

    def rank_mode(self, mode: int = -1) -> int:
        """Partition ranking on this engine's device (gk_rank_mode): mode -1 queries, 0 restores the
        device's checked default, 1 forces the ballot-match fallback.  Returns 1 if ballot-match
        ranking is in use afterwards."""
        active = ctypes.c_int(0)
        self._check(self.lib.gk_rank_mode(self.ctx, int(mode), ctypes.byref(active)))
        return active.value

    # -----------------------------------------------------------------------------------------
    def _check(self, rc: int):
        if rc != GK_OK:
            msg = self.lib.gk_last_error(self.ctx)
            raise GkError(rc, msg.decode() if msg else "")

    def set_sequence(self, sba: np.ndarray, seg_starts: np.ndarray):
        sba = np.ascontiguousarray(sba, dtype=np.uint8)
        seg = np.ascontiguousarray(seg_starts, dtype=np.uint32)
        self._check(self.lib.gk_set_sequence(self.ctx, _ptr(sba, ctypes.c_uint8), sba.size,
                                             _ptr(seg, ctypes.c_uint32), seg.size))

    def sort_hint(self, k: int):
        """gk_sort_hint: later set_sequence calls of a single-contig A/C/G/T sequence also run the
        first pass of sort(k) while the sequence streams in (0 clears)."""
        self._check(self.lib.gk_sort_hint(self.ctx, int(k or 0), 0))

    def is_acgt(self) -> bool:
        v = ctypes.c_int(0)
        self._check(self.lib.gk_alphabet_is_acgt(self.ctx, ctypes.byref(v)))
        return bool(v.value)

    def resident_packed(self) -> bool:
        """The 2-bit packed copy of the sequence is resident (gk_resident_packed)."""
        v = ctypes.c_int(0)
        self._check(self.lib.gk_resident_packed(self.ctx, ctypes.byref(v)))
        return bool(v.value)

    def enumerate(self, min_kmer_len: int) -> int:
        n = ctypes.c_uint64(0)
        self._check(self.lib.gk_enumerate(self.ctx, min_kmer_len, ctypes.byref(n)))
        self.n = n.value
        return self.n

    def copy_sequence(self, length: int) -> np.ndarray:
        """The device-resident sba (gk_copy_sequence)."""
        out = np.empty(length, dtype=np.uint8)
        self._check(self.lib.gk_copy_sequence(self.ctx, _ptr(out, ctypes.c_uint8), length))
        return out

    def set_start_indices(self, starts: np.ndarray, min_kmer_len: int):
        arr = np.ascontiguousarray(starts, dtype=np.uint32)
        self._check(self.lib.gk_set_start_indices(self.ctx, _ptr(arr, ctypes.c_uint32), arr.size, min_kmer_len))
        self.n = arr.size

    def sort(self, max_kmer_len: int = None, canonical: bool = False, quicksort_order: bool = False):
        flags = (SORT_CANONICAL if canonical else 0) | (SORT_QUICKSORT_ORDER if quicksort_order else 0)
        self._check(self.lib.gk_sort(self.ctx, 0 if max_kmer_len is None else int(max_kmer_len), flags))

    def copy_strands(self) -> np.ndarray:
        out = np.empty(self.n, dtype=np.uint8)
        self._check(self.lib.gk_copy_strands(self.ctx, _ptr(out, ctypes.c_uint8), out.size))
        return out

    def sync(self):
        self._check(self.lib.gk_sync(self.ctx))

    def copy_starts(self, out: np.ndarray = None) -> np.ndarray:
        if out is None:
            out = np.empty(self.n, dtype=np.uint32)
        self._check(self.lib.gk_copy_start_indices(self.ctx, _ptr(out, ctypes.c_uint32), self.n))
        return out

    def start_range(self, offset: int, count: int) -> np.ndarray:
        out = np.empty(count, dtype=np.uint32)
        self._check(self.lib.gk_copy_start_range(self.ctx, offset, _ptr(out, ctypes.c_uint32), count))
        return out

    def key_layout(self):
        w, b, s = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self.lib.gk_key_layout(self.ctx, ctypes.byref(w), ctypes.byref(b), ctypes.byref(s)))
        return w.value, b.value, s.value

    def copy_keys(self) -> np.ndarray:
        words, _, _ = self.key_layout()
        out = np.empty((self.n, words), dtype=np.uint64)
        self._check(self.lib.gk_copy_keys(self.ctx, _ptr(out, ctypes.c_uint64), out.size))
        return out

    def set_filter_mask(self, mask: np.ndarray):
        m = np.ascontiguousarray(mask, dtype=np.uint8)
        self._check(self.lib.gk_set_filter_mask(self.ctx, _ptr(m, ctypes.c_uint8), m.size))

    def set_group_heads(self, heads: np.ndarray):
        h = np.ascontiguousarray(heads, dtype=np.uint8)
        self._check(self.lib.gk_set_group_heads(self.ctx, _ptr(h, ctypes.c_uint8), h.size))

    def _raise_filter(self, rc, code, idx):
        if rc == GK_E_FILTER:
            raise FilterRaised(code.value, idx.value)
        self._check(rc)

    def group_hist(self, is_sorted, kmer_len, filt: GkFilter, min_group_size, max_group_size, max_counts_bin):
        hist = np.zeros(max_counts_bin + 1, dtype=np.int64)
        total = ctypes.c_int64(0)
        code, idx = ctypes.c_int32(0), ctypes.c_uint64(0)
        rc = self.lib.gk_group_hist(self.ctx, _group_mode(is_sorted), -1 if kmer_len is None else int(kmer_len),
                                    ctypes.byref(filt), int(min_group_size),
                                    -1 if max_group_size is None else int(max_group_size), int(max_counts_bin),
                                    _ptr(hist, ctypes.c_int64), ctypes.byref(total), ctypes.byref(code),
                                    ctypes.byref(idx))
        self._raise_filter(rc, code, idx)
        return hist, int(total.value)

    def group_members(self, is_sorted, kmer_len, filt: GkFilter, min_group_size, max_group_size, yield_first_n):
        args = (_group_mode(is_sorted), -1 if kmer_len is None else int(kmer_len), ctypes.byref(filt),
                int(min_group_size), -1 if max_group_size is None else int(max_group_size),
                -1 if yield_first_n is None else int(yield_first_n))
        count = ctypes.c_uint64(0)
        code, idx = ctypes.c_int32(0), ctypes.c_uint64(0)
        rc = self.lib.gk_group_members(self.ctx, *args, None, None, None, 0, ctypes.byref(count),
                                       ctypes.byref(code), ctypes.byref(idx))
        self._raise_filter(rc, code, idx)
        m = count.value
        num = np.empty(m, dtype=np.uint64)
        yld = np.empty(m, dtype=np.uint32)
        tot = np.empty(m, dtype=np.uint32)
        if m:
            rc = self.lib.gk_group_members(self.ctx, *args, _ptr(num, ctypes.c_uint64), _ptr(yld, ctypes.c_uint32),
                                           _ptr(tot, ctypes.c_uint32), m, ctypes.byref(count), ctypes.byref(code),
                                           ctypes.byref(idx))
            self._raise_filter(rc, code, idx)
        return num, yld, tot

    def unique_counts(self):
        g = ctypes.c_uint64(0)
        self._check(self.lib.gk_unique_counts(self.ctx, ctypes.byref(g)))
        starts = np.empty(g.value, dtype=np.uint64)
        counts = np.empty(g.value, dtype=np.uint32)
        self._check(self.lib.gk_copy_unique(self.ctx, _ptr(starts, ctypes.c_uint64), _ptr(counts, ctypes.c_uint32),
                                            g.value))
        return starts, counts

    def locate(self, kmer_nums: np.ndarray):
        """(start sba index, segment) of each kmer_num, on the device (gk_locate)."""
        nums = np.ascontiguousarray(kmer_nums, dtype=np.uint64)
        m = len(nums)
        sba_idx = np.empty(m, dtype=np.uint32)
        seg = np.empty(m, dtype=np.uint32)
        if m:
            self._check(self.lib.gk_locate(self.ctx, _ptr(nums, ctypes.c_uint64), m, _ptr(sba_idx, ctypes.c_uint32),
                                           _ptr(seg, ctypes.c_uint32)))
        return sba_idx, seg

    # ---- multi-GPU shards (genome_kmers.distributed) ------------------------------------------
    def shard_bucket_bits(self) -> int:
        return int(self.lib.gk_shard_bucket_bits())

    def shard_partition(self, lo: int, hi: int, k: int, keys, starts, canonical: bool = False,
                        starts_only: bool = False):
        """Encode + partition the k-mers starting in [lo, hi) into the device tensors ``keys``
        (int64) / ``starts`` (int32); returns (bucket sizes as a numpy uint64 array, count).
        starts_only (GK_SHARD_STARTS_ONLY): ``keys`` may be None, only the starts are written."""
        hist = np.zeros(1 << self.shard_bucket_bits(), dtype=np.uint64)
        n = ctypes.c_uint64(0)
        cap = starts.numel() if keys is None else min(keys.numel(), starts.numel())
        flags = (SORT_CANONICAL if canonical else 0) | (SHARD_STARTS_ONLY if starts_only else 0)
        self._check(self.lib.gk_shard_partition(self.ctx, lo, hi, k, flags, None if keys is None else keys.data_ptr(),
                                                starts.data_ptr(), cap, _ptr(hist, ctypes.c_uint64), ctypes.byref(n)))
        return hist, n.value

    def shard_sort(self, keys, starts, n: int, k: int, piece_off: np.ndarray, piece_len: np.ndarray,
                   piece_bucket: np.ndarray, canonical: bool = False, starts_only: bool = False):
        """Sort n received (key, start) pairs held in device tensors, given as bucket pieces.
        starts_only (GK_SHARD_STARTS_ONLY): ``keys`` may be None, the keys are re-derived from the
        resident sequence."""
        off = np.ascontiguousarray(piece_off, dtype=np.uint64)
        ln = np.ascontiguousarray(piece_len, dtype=np.uint64)
        bk = np.ascontiguousarray(piece_bucket, dtype=np.uint32)
        flags = (SORT_CANONICAL if canonical else 0) | (SHARD_STARTS_ONLY if starts_only else 0)
        self._check(self.lib.gk_shard_sort(self.ctx, keys.data_ptr() if n and keys is not None else None,
                                           starts.data_ptr() if n else None, n, k, flags, _ptr(off, ctypes.c_uint64),
                                           _ptr(ln, ctypes.c_uint64), _ptr(bk, ctypes.c_uint32), len(bk)))
        self.n = n

    def shard_histogram(self, lo: int, hi: int, k: int, canonical: bool = False):
        """Top-digit histogram of the k-mers starting in [lo, hi): (numpy uint64[1 << bits], bits)."""
        hist = np.zeros(4096, dtype=np.uint64)
        bits = ctypes.c_uint32(0)
        self._check(self.lib.gk_shard_histogram(self.ctx, lo, hi, k, SORT_CANONICAL if canonical else 0,
                                                _ptr(hist, ctypes.c_uint64), ctypes.byref(bits)))
        return hist[:1 << bits.value].copy(), bits.value

    def shard_class_b(self, lo: int, hi: int, k: int, hist: np.ndarray, canonical: bool = False):
        """Class-B k-mers starting in [lo, hi) (gk_shard_class_b): (non-homopolymer starts uint32[m],
        homopolymer runs uint32[r, 3] = (first start, count, letter)); their ownership bins are added
        to ``hist`` (uint64, gk_shard_histogram's bins) in place.  ACGT-only sba: two empty arrays."""
        full = np.zeros(4096, dtype=np.uint64)
        full[:len(hist)] = hist
        nr, nh = ctypes.c_uint64(0), ctypes.c_uint64(0)
        self._check(self.lib.gk_shard_class_b(self.ctx, lo, hi, k, SORT_CANONICAL if canonical else 0,
                                              _ptr(full, ctypes.c_uint64), ctypes.byref(nr), ctypes.byref(nh)))
        hist[:] = full[:len(hist)]
        rest = np.empty(nr.value, dtype=np.uint32)
        runs = np.empty((nh.value, 3), dtype=np.uint32)
        self._check(self.lib.gk_shard_class_b_copy(self.ctx, _ptr(rest, ctypes.c_uint32), nr.value,
                                                   _ptr(runs, ctypes.c_uint32), nh.value))
        return rest, runs

    def shard_sort_range_b(self, k: int, digit_lo: int, digit_hi: int, rest: np.ndarray, runs: np.ndarray,
                           canonical: bool = False) -> int:
        """shard_sort_range with the class-B k-mers of the whole sba given (every rank's
        shard_class_b lists concatenated in rank order) instead of scanned for."""
        rest = np.ascontiguousarray(rest, dtype=np.uint32)
        runs = np.ascontiguousarray(runs, dtype=np.uint32).reshape(-1, 3)
        n = ctypes.c_uint64(0)
        self._check(self.lib.gk_shard_sort_range_b(self.ctx, k, SORT_CANONICAL if canonical else 0, digit_lo,
                                                   digit_hi, _ptr(rest, ctypes.c_uint32), len(rest),
                                                   _ptr(runs, ctypes.c_uint32), len(runs), ctypes.byref(n)))
        self.n = n.value
        return n.value

    def shard_sort_range(self, k: int, digit_lo: int, digit_hi: int, canonical: bool = False) -> int:
        """Sort the k-mers of the whole sequence whose top digit is in [digit_lo, digit_hi); returns
        their number (the context then holds them as after sort(k))."""
        n = ctypes.c_uint64(0)
        self._check(self.lib.gk_shard_sort_range(self.ctx, k, SORT_CANONICAL if canonical else 0, digit_lo, digit_hi,
                                                 ctypes.byref(n)))
        self.n = n.value
        return n.value

    def unique_count_only(self) -> int:
        g = ctypes.c_uint64(0)
        self._check(self.lib.gk_unique_counts(self.ctx, ctypes.byref(g)))
        return g.value

    def device_views(self):
        s, k, n, w = _P(), _P(), ctypes.c_uint64(), ctypes.c_uint32()
        self._check(self.lib.gk_device_views(self.ctx, ctypes.byref(s), ctypes.byref(k), ctypes.byref(n),
                                             ctypes.byref(w)))
        return s.value, k.value, n.value, w.value

    def device_unique(self):
        """(device group starts u32*, device counts u32*, n_unique) of the last unique_counts."""
        g, c, n = _P(), _P(), ctypes.c_uint64()
        self._check(self.lib.gk_device_unique(self.ctx, ctypes.byref(g), ctypes.byref(c), ctypes.byref(n)))
        return g.value, c.value, n.value

    def materialize_keys(self) -> int:
        """Make the sorted keys resident (re-encoded from the sorted starts if the sort left them
        stale); returns the key words per k-mer."""
        s, k, n, w = _P(), _P(), ctypes.c_uint64(), ctypes.c_uint32()
        self._check(self.lib.gk_device_views(self.ctx, ctypes.byref(s), ctypes.byref(k), ctypes.byref(n),
                                             ctypes.byref(w)))
        return w.value

    def device_starts(self):
        """(device pointer of the current start indices, n) -- no key materialisation."""
        s, n = _P(), ctypes.c_uint64()
        self._check(self.lib.gk_device_views(self.ctx, ctypes.byref(s), None, ctypes.byref(n), None))
        return s.value, n.value

    def stream_handle(self) -> int:
        s = _P()
        self._check(self.lib.gk_stream(self.ctx, ctypes.byref(s)))
        return s.value or 0

    def profile_enable(self, on: bool = True):
        self._check(self.lib.gk_profile_enable(self.ctx, int(on)))

    def profile_report(self) -> dict:
        import json

        buf = ctypes.create_string_buffer(1 << 16)
        self._check(self.lib.gk_profile_report(self.ctx, buf, len(buf)))
        return json.loads(buf.value.decode())
