"""Kmers -- drop-in for mrperkett/genome-kmers ``genome_kmers/kmers.py`` (v1.0.1) on MI355X.

The class surface (constructor, members, ``sort``, ``get_kmers``, ``get_kmer_count``,
``get_kmer_group_counts``, ``get_kmer_str``, the module-level comparators / filters / group
helpers) keeps the reference's names, argument meaning, error types and messages.  The work is
done by libgkm.so on the GPU (``_native.Engine``):

  enumerate   Kmers._initialize_single_pass (kmers.py:789-861)      -> gk_enumerate
  sort        Kmers.sort (kmers.py:1624-1731), numba quicksort        -> gk_sort (radix / doubling)
  groups      kmer_info_by_group_generator / get_kmer_group_size_hist
              (kmers.py:454-648) behind get_kmers / get_kmer_count /
              get_kmer_group_counts (kmers.py:869-1178)               -> gk_group_hist / gk_group_members

There is no CPU fallback for any of these.  Tie order: equal k-mers come out ordered by start
index -- the reference's ``get_is_less_than_func(break_ties=True)`` order (kmers.py:1710-1711).
The reference's default ``sort()`` leaves ties in numba-quicksort order, which no parallel sort
reproduces; sorted k-mers, group sizes and counts are identical either way.

The scalar helpers (``compare_sba_kmers_lexicographically``, the filter callables, ...) are kept
as host functions for API compatibility; when a built-in filter or comparator is handed to a
``Kmers`` method it is recognised and executed on the device instead.
"""

import shelve
from pathlib import Path
from typing import Callable, Generator, Union

import numpy as np

from . import _native
from .sequence_collection import SequenceCollection

DOLLAR = ord("$")


# ---------------------------------------------------------------------------------------------
# filters (kmers.py:14-259): host-callable with the reference signature, plus a device spec
# ---------------------------------------------------------------------------------------------
class _DeviceFilter:
    """A built-in filter: callable as ``f(sba, sba_strand, kmer_sba_start_idx) -> bool`` and
    carrying the gk_filter record the device evaluates."""

    def __init__(self, kind: int, fn: Callable, p0: int = 0, p1: int = 0, p2: int = 0, kmer_len: int = None):
        self.kind = kind
        self._fn = fn
        self.params = (int(p0), int(p1), int(p2))
        self.kmer_len = kmer_len

    def __call__(self, sba, sba_strand, kmer_sba_start_idx):
        return self._fn(sba, sba_strand, kmer_sba_start_idx)

    def gk_filter(self) -> _native.GkFilter:
        return _native.GkFilter(self.kind, 0, *self.params)


def _keep_all(sba, sba_strand, kmer_sba_start_idx):
    return True


kmer_filter_keep_all = _DeviceFilter(_native.FILTER_KEEP_ALL, _keep_all)


def gen_kmer_length_filter_func(min_kmer_len: int) -> Callable:
    """Pass if the k-mer has min_kmer_len bases before '$' (kmers.py:19-34)."""

    def filt(sba, sba_strand, kmer_sba_start_idx):
        return kmer_has_required_len(sba, kmer_sba_start_idx, min_kmer_len)

    return _DeviceFilter(_native.FILTER_LENGTH, filt, min_kmer_len)


def gen_kmer_homopolymer_filter_func(max_homopolymer_size: int, kmer_len: int) -> Callable:
    """Pass if no homopolymer is longer than max_homopolymer_size (kmers.py:37-100)."""
    if max_homopolymer_size < 1:
        raise ValueError(f"max_homopolymer_size ({max_homopolymer_size}) must be >= 1")
    if kmer_len < 1:
        raise ValueError(f"kmer_len ({kmer_len}) must be >= 1")

    def filt(sba, sba_strand, kmer_sba_start_idx):
        if kmer_sba_start_idx + kmer_len - 1 >= len(sba):
            raise ValueError(
                f"The kmer_len ({kmer_len}) requested is too large for kmer_sba_start_idx ({kmer_sba_start_idx})"
            )
        if kmer_len < max_homopolymer_size:
            return True
        size = 1
        for k in range(1, kmer_len):
            i = kmer_sba_start_idx + k
            if sba[i] == DOLLAR:
                raise ValueError(
                    f"The kmer_len ({kmer_len}) requested is too large for kmer_sba_start_idx ({kmer_sba_start_idx})"
                )
            if sba[i] == sba[i - 1]:
                size += 1
                if size > max_homopolymer_size:
                    return False
            else:
                size = 1
        return True

    return _DeviceFilter(_native.FILTER_HOMOPOLYMER, filt, max_homopolymer_size, kmer_len, kmer_len=kmer_len)


def gen_kmer_gc_content_filter_func(min_allowed_gc_frac: float, max_allowed_gc_frac: float, kmer_len: int) -> Callable:
    """Pass if the GC fraction lies in [min, max] (kmers.py:103-192)."""
    if min_allowed_gc_frac > max_allowed_gc_frac:
        raise ValueError(
            f"min_allowed_gc_frac ({min_allowed_gc_frac}) must be <= max_allowed_gc_frac ({max_allowed_gc_frac})"
        )
    if min_allowed_gc_frac < 0.0 or min_allowed_gc_frac > 1.0:
        raise ValueError(f"min_allowed_gc_frac ({min_allowed_gc_frac}) must be in the range [0.0, 1.0]")
    if max_allowed_gc_frac < 0.0 or max_allowed_gc_frac > 1.0:
        raise ValueError(f"max_allowed_gc_frac ({max_allowed_gc_frac}) must be in the range [0.0, 1.0]")
    min_count = int(np.ceil(kmer_len * min_allowed_gc_frac))
    max_count = int(np.floor(kmer_len * max_allowed_gc_frac))

    def filt(sba, sba_strand, kmer_sba_start_idx):
        if max_count < min_count:
            return False
        gc = 0
        for k in range(kmer_len):
            base = sba[kmer_sba_start_idx + k]
            if base == DOLLAR:
                raise ValueError(
                    f"The kmer_len ({kmer_len}) requested is too larger for kmer_sba_start_idx ({kmer_sba_start_idx})"
                )
            if base == 71 or base == 67:
                gc += 1
                if gc > max_count:
                    return False
        return min_count <= gc <= max_count

    return _DeviceFilter(_native.FILTER_GC, filt, min_count, max_count, kmer_len, kmer_len=kmer_len)


def gen_no_ambiguous_bases_filter(kmer_len: int) -> Callable:
    """Pass if the k-mer holds only A, T, G, C (kmers.py:195-229)."""

    def no_ambiguous_bases_filter(sba, sba_strand, kmer_sba_start_idx):
        if kmer_sba_start_idx + kmer_len > len(sba):
            raise ValueError(f"kmer_len ({kmer_len}) is invalid. It extends beyond len(sba)")
        for k in range(kmer_len):
            base = sba[kmer_sba_start_idx + k]
            if base == 36:
                raise ValueError(f"end of segment was reached. kmer_len ({kmer_len}) invalid.")
            if base not in (65, 84, 71, 67):
                return False
        return True

    return _DeviceFilter(_native.FILTER_NO_AMBIGUOUS, no_ambiguous_bases_filter, kmer_len, kmer_len=kmer_len)


def _crispr_ngg(sba, sba_strand, kmer_sba_start_idx) -> bool:
    if kmer_sba_start_idx + 23 > len(sba):
        raise ValueError("The guide defined at this start index extends beyond the sba")
    return bool(sba[kmer_sba_start_idx + 21] == 71 and sba[kmer_sba_start_idx + 22] == 71)


crispr_ngg_pam_filter = _DeviceFilter(_native.FILTER_CRISPR_NGG, _crispr_ngg)


def kmer_has_required_len(sba: np.ndarray, sba_start_idx: int, min_kmer_len: int) -> bool:
    """True if min_kmer_len bases precede '$' / the end (kmers.py:262-282)."""
    for idx in range(sba_start_idx, sba_start_idx + min_kmer_len):
        if idx >= len(sba) or sba[idx] == DOLLAR:
            return False
    return True


# ---------------------------------------------------------------------------------------------
# comparators (kmers.py:285-397)
# ---------------------------------------------------------------------------------------------
def compare_sba_kmers_lexicographically(sba_a, sba_b, kmer_sba_start_idx_a, kmer_sba_start_idx_b,
                                        max_kmer_len: Union[int, None] = None) -> tuple:
    """Three-way compare of two k-mers by ASCII bytes; '$' / end of array is smaller than any base.

    Returns (comparison, last_kmer_index_compared); see kmers.py:306-397.
    """
    k = 0
    while True:
        ia = kmer_sba_start_idx_a + k
        ib = kmer_sba_start_idx_b + k
        oa = ia >= len(sba_a) or sba_a[ia] == DOLLAR
        ob = ib >= len(sba_b) or sba_b[ib] == DOLLAR
        if oa or ob:
            last = k - 1
            if last < 0:
                raise AssertionError("There were no valid kmer bases to compare")
            if oa and not ob:
                return -1, last
            if ob and not oa:
                return 1, last
            return 0, last
        if sba_a[ia] < sba_b[ib]:
            return -1, k
        if sba_a[ia] > sba_b[ib]:
            return 1, k
        if max_kmer_len is not None and k == max_kmer_len - 1:
            return 0, k
        k += 1


class _Comparator:
    """compare_sba_kmers_lexicographically bound to a kmer_len; recognised by the device path."""

    def __init__(self, kmer_len, always_less=False):
        self.kmer_len = kmer_len
        self.always_less = always_less

    def __call__(self, sba_a, sba_b, kmer_sba_start_idx_a, kmer_sba_start_idx_b, max_kmer_len=None):
        if self.always_less:
            return -1, 0
        return compare_sba_kmers_lexicographically(sba_a, sba_b, kmer_sba_start_idx_a, kmer_sba_start_idx_b,
                                                   max_kmer_len=self.kmer_len)


def get_compare_sba_kmers_func(kmer_len):
    """Comparator with max_kmer_len = kmer_len (kmers.py:285-292)."""
    return _Comparator(kmer_len)


compare_sba_kmers_always_less_than = _Comparator(None, always_less=True)


# ---------------------------------------------------------------------------------------------
# group helpers (kmers.py:400-648)
# ---------------------------------------------------------------------------------------------
def get_kmer_info_minimal(kmer_num, kmer_sba_start_indices, sba, kmer_len, group_size_yielded, group_size_total):
    """(kmer_num, group_size_yielded, group_size_total) -- kmers.py:400-425"""
    return kmer_num, group_size_yielded, group_size_total


def get_kmer_info_group_size_only(kmer_num, kmer_sba_start_indices, sba, kmer_len, group_size_yielded,
                                  group_size_total):
    """group_size_total -- kmers.py:428-451"""
    return group_size_total


def _check_group_args(min_group_size, max_group_size, yield_first_n):
    # kmers.py:565-573
    if min_group_size < 1:
        raise ValueError(f"min_group_size ({min_group_size}) must be >= 1")
    if max_group_size is not None and max_group_size < min_group_size:
        raise ValueError(
            f"if max_group_size ({max_group_size}) is specified, it must be >= min_group_size ({min_group_size})"
        )
    if yield_first_n is not None and yield_first_n < 1:
        raise ValueError(f"if yield_first_n ({yield_first_n}) is specified, it must be > 0")


def _filter_error(ferr: int, sba_idx: int, filt) -> Exception:
    """Rebuild the exception the reference's filter raises (kmers.py:66-69, 176-179, 212-221, 252-253)."""
    k = getattr(filt, "kmer_len", None)
    if ferr == _native.FERR_HOMO_LEN:
        return ValueError(f"The kmer_len ({k}) requested is too large for kmer_sba_start_idx ({sba_idx})")
    if ferr == _native.FERR_GC_LEN:
        return ValueError(f"The kmer_len ({k}) requested is too larger for kmer_sba_start_idx ({sba_idx})")
    if ferr == _native.FERR_GC_OOB:
        return IndexError(f"kmer at sba index {sba_idx} of length {k} extends beyond len(sba)")
    if ferr == _native.FERR_AMBIG_LEN:
        return ValueError(f"kmer_len ({k}) is invalid. It extends beyond len(sba)")
    if ferr == _native.FERR_AMBIG_SEG:
        return ValueError(f"end of segment was reached. kmer_len ({k}) invalid.")
    if ferr == _native.FERR_CRISPR_LEN:
        return ValueError("The guide defined at this start index extends beyond the sba")
    return RuntimeError(f"device filter error {ferr} at sba index {sba_idx}")


def _device_filter(engine: "_native.Engine", filt, sba, sba_strand, starts_fn) -> _native.GkFilter:
    """gk_filter for a built-in filter; a custom Python callable is evaluated once per k-mer on the
    host (it is user code) into a mask that the device consumes."""
    if isinstance(filt, _DeviceFilter):
        return filt.gk_filter()
    if not callable(filt):
        raise TypeError("kmer_filter_func must be callable")
    starts = starts_fn()
    mask = np.fromiter((bool(filt(sba, sba_strand, int(s))) for s in starts), dtype=np.uint8, count=len(starts))
    engine.set_filter_mask(mask)
    return _native.GkFilter(_native.FILTER_MASK, 0, 0, 0, 0)


def _comparator_mode(cmp) -> tuple:
    """(is_sorted, kmer_len) for a recognised comparator; (None, None) for a custom one."""
    if isinstance(cmp, _Comparator):
        return (not cmp.always_less), cmp.kmer_len
    if not callable(cmp):
        raise TypeError("kmer_comparison_func must be callable")
    return None, None


def _custom_groups(engine: "_native.Engine", cmp, filt, sba, sba_strand, starts) -> _native.GkFilter:
    """A custom ``kmer_comparison_func`` (user code: the device cannot run it) decides the groups on
    the host, as the reference's generator does (kmers.py:579-601): each k-mer that passes the
    filter is compared with the previous one that passed, ``comparison == 0`` meaning the same
    group.  The filter runs on the host too, so that filter and comparator are called in the
    reference's order and the first raise is the reference's.  The device then runs the group
    pass over the resulting head mask (gk_set_group_heads); returns the filter spec to pass."""
    starts = np.asarray(starts)
    keep_all = isinstance(filt, _DeviceFilter) and filt.kind == _native.FILTER_KEEP_ALL
    if not keep_all and not callable(filt):
        raise TypeError("kmer_filter_func must be callable")
    valid = np.ones(len(starts), dtype=np.uint8)
    heads = np.zeros(len(starts), dtype=np.uint8)
    prev = None
    for i, s in enumerate(starts.tolist()):
        if not keep_all and not filt(sba, sba_strand, s):
            valid[i] = 0
            continue
        if prev is not None:
            comparison, _ = cmp(sba, sba, prev, s)
            heads[i] = comparison != 0
        prev = s
    engine.set_group_heads(heads)
    if keep_all:
        return filt.gk_filter()
    engine.set_filter_mask(valid)
    return _native.GkFilter(_native.FILTER_MASK, 0, 0, 0, 0)


def _engine_for_arrays(sba: np.ndarray, kmer_start_indices: np.ndarray) -> "_native.Engine":
    sba = np.ascontiguousarray(sba, dtype=np.uint8)
    seg = np.concatenate([[0], np.flatnonzero(sba == DOLLAR) + 1]).astype(np.uint32)
    eng = _native.Engine()
    eng.set_sequence(sba, seg)
    eng.set_start_indices(np.asarray(kmer_start_indices, dtype=np.uint32), 1)
    return eng


def get_kmer_group_size_hist(sba, sba_strand, kmer_len, kmer_start_indices, kmer_comparison_func, kmer_filter_func,
                             min_group_size: int = 1, max_group_size: Union[int, None] = None,
                             max_counts_bin: int = 1000000) -> tuple:
    """Histogram of group sizes and total k-mer count (kmers.py:454-520), on the device."""
    if max_counts_bin <= 0:
        raise ValueError(f"max_counts_bin ({max_counts_bin}) must be >= 1")
    _check_group_args(min_group_size, max_group_size, 1)
    is_sorted, cmp_len = _comparator_mode(kmer_comparison_func)
    if len(kmer_start_indices) == 0:
        return np.zeros(max_counts_bin + 1, dtype=np.int64), 0
    eng = _engine_for_arrays(sba, kmer_start_indices)
    if is_sorted is None:  # custom comparator: groups decided on the host, counted on the device
        filt = _custom_groups(eng, kmer_comparison_func, kmer_filter_func, sba, sba_strand, kmer_start_indices)
        return eng.group_hist(_native.GROUPS_FROM_HEADS, None, filt, min_group_size, max_group_size, max_counts_bin)
    filt = _device_filter(eng, kmer_filter_func, sba, sba_strand, lambda: kmer_start_indices)
    try:
        return eng.group_hist(is_sorted, cmp_len, filt, min_group_size, max_group_size, max_counts_bin)
    except _native.FilterRaised as e:
        raise _filter_error(e.ferr, e.sba_idx, kmer_filter_func) from None


def kmer_info_by_group_generator(sba, sba_strand, kmer_len, kmer_start_indices, kmer_comparison_func,
                                 kmer_filter_func, kmer_info_func, min_group_size: int = 1,
                                 max_group_size: Union[int, None] = None,
                                 yield_first_n: Union[int, None] = None) -> Generator[tuple, None, None]:
    """Yield kmer_info_func(...) for the first yield_first_n members of every group whose size lies
    in [min_group_size, max_group_size] (kmers.py:523-648); groups are computed on the device."""
    _check_group_args(min_group_size, max_group_size, yield_first_n)
    is_sorted, cmp_len = _comparator_mode(kmer_comparison_func)
    if len(kmer_start_indices) == 0:
        return
    eng = _engine_for_arrays(sba, kmer_start_indices)
    if is_sorted is None:  # custom comparator: groups decided on the host, members on the device
        filt = _custom_groups(eng, kmer_comparison_func, kmer_filter_func, sba, sba_strand, kmer_start_indices)
        nums, yielded, totals = eng.group_members(_native.GROUPS_FROM_HEADS, None, filt, min_group_size,
                                                  max_group_size, yield_first_n)
    else:
        filt = _device_filter(eng, kmer_filter_func, sba, sba_strand, lambda: kmer_start_indices)
        try:
            nums, yielded, totals = eng.group_members(is_sorted, cmp_len, filt, min_group_size, max_group_size,
                                                      yield_first_n)
        except _native.FilterRaised as e:
            raise _filter_error(e.ferr, e.sba_idx, kmer_filter_func) from None
    for num, y, t in zip(nums.tolist(), yielded.tolist(), totals.tolist()):
        yield kmer_info_func(num, kmer_start_indices, sba, kmer_len, y, t)


# ---------------------------------------------------------------------------------------------
# Kmers
# ---------------------------------------------------------------------------------------------
_UNSORTED_GROUP_MSG = (
    "Returning group parameters is not supported when kmers has not been"
    " sorted. {name} ({value}) cannot be specified. Did you"
    " mean to run sort() before getting kmers?"
)


class Kmers:
    """Memory-efficient k-mer calculations on a genome, resident on one MI355X."""

    # fixed-length Kmers run the first pass of the forward sort while the sequence is transferred
    # (gk_sort_hint); False skips it (see _get_engine for its cost)
    sort_prefetch = True

    def __init__(self, seq_coll: Union[SequenceCollection, None] = None, min_kmer_len: int = 1,
                 max_kmer_len: Union[int, None] = None, source_strand: str = "forward",
                 track_strands_separately: bool = False, method: str = "single_pass") -> None:
        # kmers.py:688-713 (same order of checks, same messages)
        if track_strands_separately:
            raise NotImplementedError(
                f"This function has not been implemented for track_strands_separately = '{track_strands_separately}'"
            )
        if source_strand != "forward":
            raise NotImplementedError(f"This function has not been implemented for source_strand = '{source_strand}'")
        if source_strand not in ("forward", "reverse_complement", "both"):
            raise ValueError(f"source_strand ({source_strand}) not recognized")
        if source_strand != "both" and track_strands_separately:
            raise ValueError(
                f"track_strands_separately can only be true if source_strand is 'both', but it is '{source_strand}'"
            )
        if min_kmer_len < 1:
            raise ValueError(f"min_kmer_len ({min_kmer_len}) must be greater than zero")
        if max_kmer_len is not None:
            if max_kmer_len < 1:
                raise ValueError(f"max_kmer_len ({max_kmer_len}) must be greater than zero")
            if min_kmer_len is not None and max_kmer_len < min_kmer_len:
                raise ValueError(f"max_kmer_len ({max_kmer_len}) is less than min_kmer_len ({min_kmer_len})")

        self.min_kmer_len = min_kmer_len
        self.max_kmer_len = max_kmer_len
        self.kmer_source_strand = source_strand
        self.track_strands_separately = track_strands_separately
        self._is_initialized = False
        self._is_set = False
        self._is_sorted = False
        self._canonical = False       # sorted by canonical k-mer (sort(canonical=True); no reference counterpart)
        self._engine = None
        self._host_starts = None      # host view of the start indices (or a user-assigned array)
        self._host_valid = True       # _host_starts matches the device order
        self._device_stale = False    # a user-assigned array has not been uploaded yet

        if seq_coll is None:
            return

        # kmers.py:730-754
        min_seq_len = None
        num_records = 0
        for _, b, e in seq_coll.iter_records():
            seq_length = e - b + 1
            if min_seq_len is None or seq_length < min_seq_len:
                min_seq_len = seq_length
            num_records += 1
        if num_records == 0:
            raise ValueError("sequence_collection is empty")
        if min_kmer_len is not None and min_kmer_len > min_seq_len:
            raise ValueError(f"min_kmer_len ({min_kmer_len}) must be <= the shortest sequence length ({min_seq_len})")
        if seq_coll.strands_loaded() != source_strand:
            raise ValueError(
                f"source_strand ({source_strand}) does not match sequence_collection loaded strand "
                f"({seq_coll.strands_loaded()})"
            )
        self.seq_coll = seq_coll
        self._initialize(method=method)

    # ---- initialisation (kmers.py:762-861) ---------------------------------------------------
    def _initialize(self, kmer_filters=[], method: str = "single_pass"):
        if kmer_filters != []:
            raise NotImplementedError("kmer_filters have not been implemented")
        if method == "double_pass":
            raise NotImplementedError(f"method '{method}' has not been implemented")
        elif method == "single_pass":
            self._initialize_single_pass(kmer_filters=kmer_filters)
        else:
            raise ValueError(f"method '{method}' not recognized")
        self._is_initialized = True

    def _initialize_single_pass(self, kmer_filters=[]):
        if kmer_filters != []:
            raise NotImplementedError("kmer_filters have not been implemented")
        num_kmers = self._get_unfiltered_kmer_count()
        if num_kmers > 2**32 - 1:
            raise NotImplementedError("the size of the required kmers array exceeds the limit set by a uint32")
        eng = self._get_engine()
        n = eng.enumerate(self.min_kmer_len)
        if n != num_kmers:
            raise AssertionError(f"logic error: last_filled_index ({n - 1}) != num_kmers - 1 ({num_kmers - 1})")
        self._host_starts = None
        self._host_valid = False
        self._device_stale = False

    def _get_unfiltered_kmer_count(self) -> int:
        num_kmers = 0
        num_records = 0
        for _, b, e in self.seq_coll.iter_records():
            num_kmers += (e - b + 1) - self.min_kmer_len + 1
            num_records += 1
        if num_records == 0:
            raise ValueError("SequenceCollection does not have any records")
        return num_kmers

    def _get_engine(self) -> "_native.Engine":
        if self._engine is None:
            eng = _native.Engine()
            # a fixed k-mer length: the transfer also runs the first pass of sort(k) (gk_sort_hint).
            # That pass costs device memory for every position (~13 B) and its work at load time;
            # a canonical, reference-order or unsorted workflow drops it, so such callers can set
            # Kmers.sort_prefetch = False (class- or instance-wide) before the first device call
            if self.sort_prefetch and self.min_kmer_len is not None and self.min_kmer_len == self.max_kmer_len:
                eng.sort_hint(self.min_kmer_len)
            eng.set_sequence(self.seq_coll.forward_sba, self.seq_coll._forward_sba_seg_starts)
            self._engine = eng
        return self._engine

    # ---- start indices: device-resident, host view on demand ---------------------------------
    @property
    def kmer_sba_start_indices(self):
        if not self._host_valid and self._engine is not None:
            n = self._engine.n
            buf = self._host_starts
            if buf is None or buf.shape != (n,) or buf.dtype != np.uint32 or not buf.flags.c_contiguous:
                buf = np.empty(n, dtype=np.uint32)
            writeable = buf.flags.writeable
            buf.setflags(write=True)
            self._engine.copy_starts(buf)
            buf.setflags(write=writeable)
            self._host_starts = buf
            self._host_valid = True
        return self._host_starts

    @kmer_sba_start_indices.setter
    def kmer_sba_start_indices(self, value):
        self._canonical = False
        self._host_starts = value
        self._host_valid = True
        self._device_stale = True

    def _sync_device(self):
        """Upload a user-assigned start array before device work."""
        if self._device_stale:
            if self._host_starts is None:
                raise TypeError("kmer_sba_start_indices is None")
            self._get_engine().set_start_indices(np.asarray(self._host_starts, dtype=np.uint32), self.min_kmer_len)
            self._device_stale = False
            if self._canonical and self._is_sorted:
                # a canonical order loaded from a file: the device re-derives its canonical sorted
                # state (the same order: equal canonical k-mers are in start order either way)
                self._engine.sort(self.max_kmer_len, canonical=True)
        if self._engine is None:
            raise TypeError("Kmers has no sequence collection / k-mers")

    def _after_device_reorder(self):
        """Keep the reference's in-place semantics for a host array the caller already holds."""
        buf = self._host_starts
        if buf is not None and isinstance(buf, np.ndarray) and buf.dtype == np.uint32 and buf.flags.writeable \
                and buf.flags.c_contiguous and buf.shape == (self._engine.n,):
            self._engine.copy_starts(buf)
            self._host_valid = True
        else:
            self._host_valid = False

    def __len__(self):
        if self._engine is not None and not self._device_stale:
            return self._engine.n
        return len(self.kmer_sba_start_indices)

    def __getitem__(self):
        pass

    def _num_kmers(self) -> int:
        return len(self)

    def _check_forward(self):
        if self.kmer_source_strand != "forward" or self.seq_coll.strands_loaded() != "forward":
            raise NotImplementedError(
                f"both kmer_source_strand ({self.kmer_source_strand}) and "
                "sequence_collection.strands_loaded() must be 'forward'"
            )

    def _check_canonical_len(self, kmer_len):
        if self._is_sorted and getattr(self, "_canonical", False) and kmer_len != self.max_kmer_len:
            raise ValueError(f"canonical k-mers are grouped at kmer_len == {self.max_kmer_len} only "
                             f"(kmer_len = {kmer_len})")

    def _check_unsorted_group_args(self, min_group_size, max_group_size, yield_first_n=None):
        if not self._is_sorted:
            if min_group_size != 1:
                raise ValueError(_UNSORTED_GROUP_MSG.format(name="min_group_size", value=min_group_size))
            if max_group_size is not None:
                raise ValueError(_UNSORTED_GROUP_MSG.format(name="max_group_size", value=max_group_size))
            if yield_first_n is not None:
                raise ValueError(_UNSORTED_GROUP_MSG.format(name="yield_first_n", value=yield_first_n))

    def _filter_spec(self, filt):
        return _device_filter(self._engine, filt, self.seq_coll.forward_sba, self.seq_coll.strands_loaded(),
                              lambda: self.kmer_sba_start_indices)

    # ---- queries (kmers.py:869-1178) ---------------------------------------------------------
    def get_kmers(self, kmer_len: Union[int, None], one_based_seq_index: bool = False,
                  kmer_filter_func: Callable = kmer_filter_keep_all, kmer_info_to_yield: str = "minimum",
                  min_group_size: int = 1, max_group_size: Union[int, None] = None,
                  yield_first_n: Union[int, None] = None) -> Generator[tuple, None, None]:
        """Yield k-mer info for qualifying groups (kmers.py:869-992); groups computed on the GPU."""
        self._check_forward()
        if kmer_len is not None and kmer_len < 1:
            raise ValueError(f"kmer_len ({kmer_len}) must be > 0")
        self._check_unsorted_group_args(min_group_size, max_group_size, yield_first_n)
        self._check_canonical_len(kmer_len)
        if kmer_info_to_yield not in ("minimum", "full"):
            raise ValueError(f"kmer_info_to_yield ({kmer_info_to_yield}) not recognized")
        _check_group_args(min_group_size, max_group_size, yield_first_n)
        self._sync_device()
        if self._engine.n == 0:
            return
        filt = self._filter_spec(kmer_filter_func)
        try:
            nums, yielded, totals = self._engine.group_members(self._is_sorted, kmer_len, filt, min_group_size,
                                                               max_group_size, yield_first_n)
        except _native.FilterRaised as e:
            raise _filter_error(e.ferr, e.sba_idx, kmer_filter_func) from None
        if kmer_info_to_yield == "minimum":
            for t in zip(nums.tolist(), yielded.tolist(), totals.tolist()):
                yield t
            return
        yield from self._full_info(nums, yielded, totals, kmer_len, one_based_seq_index)

    def _full_info(self, nums, yielded, totals, kmer_len, one_based):
        """get_kmer_info (kmers.py:1180-1264) for every yielded k-mer at once: the starts and their
        segments come from the device (gk_locate), the rest is vectorised here; a k-mer whose
        kmer_len runs past its segment raises at its turn, as the reference's generator does."""
        sc = self.seq_coll
        sba_strand = sc._get_sba_strand_to_use(sc.strands_loaded())
        sba, seg_starts, names = sc._strand_arrays(sba_strand)
        strand_char = "+" if sba_strand == "forward" else "-"
        sba_idx, seg = self._engine.locate(nums)
        starts64 = seg_starts.astype(np.int64)
        b = starts64[seg]
        e = np.where(seg == len(seg_starts) - 1, len(sba) - 1, starts64[np.minimum(seg + 1, len(seg_starts) - 1)] - 2)
        s64 = sba_idx.astype(np.int64)
        seq_idx = (s64 - b if sba_strand == "forward" else e - s64) + (1 if one_based else 0)
        klen = (e - s64 + 1) if kmer_len is None else np.full(len(s64), kmer_len, dtype=np.int64)
        bad = (s64 > e) | ((s64 + klen - 1) > e)
        first_bad = int(np.argmax(bad)) if bad.any() else len(s64)
        names = tuple(names)
        num_l, y_l, t_l, seg_l, seq_l, k_l = (nums.tolist(), yielded.tolist(), totals.tolist(), seg.tolist(),
                                              seq_idx.tolist(), klen.tolist())
        for i in range(first_bad):
            yield (num_l[i], strand_char, names[seg_l[i]], seq_l[i], k_l[i], y_l[i], t_l[i])
        if first_bad < len(s64):  # the reference's own checks and messages for that k-mer
            info = self.generate_get_kmer_info_func(one_based)
            i = first_bad
            yield info(num_l[i], self._start_lookup(num_l[i]), sba, kmer_len, y_l[i], t_l[i])

    def _start_lookup(self, kmer_num):
        """A one-element start view for generate_get_kmer_info_func's checks."""

        class _One:
            def __len__(_self):
                return int(self._engine.n)

            def __getitem__(_self, k):
                return int(self._engine.locate(np.array([k], dtype=np.uint64))[0][0])

        return _One()

    def get_kmer_count(self, kmer_len: Union[int, None], kmer_filter_func: Callable = kmer_filter_keep_all,
                       min_group_size: int = 1, max_group_size: Union[int, None] = None) -> int:
        """Total k-mers in qualifying groups (kmers.py:994-1083), on the GPU."""
        self._check_forward()
        if kmer_len is not None and kmer_len < 1:
            raise ValueError(f"kmer_len ({kmer_len}) must be > 0")
        self._check_unsorted_group_args(min_group_size, max_group_size)
        self._check_canonical_len(kmer_len)
        _, total = self._group_hist(kmer_len, kmer_filter_func, min_group_size, max_group_size, 1000000)
        return total

    def get_kmer_group_counts(self, kmer_len: Union[int, None], kmer_filter_func: Callable = kmer_filter_keep_all,
                              min_group_size: int = 1, max_group_size: Union[int, None] = None,
                              max_counts_bin: int = 1000000) -> tuple:
        """Histogram of group sizes + total (kmers.py:1085-1178), on the GPU."""
        self._check_forward()
        if kmer_len is not None and kmer_len < 1:
            raise ValueError(f"kmer_len ({kmer_len}) must be > 0")
        self._check_unsorted_group_args(min_group_size, max_group_size)
        self._check_canonical_len(kmer_len)
        if not self._is_sorted:
            raise AssertionError("The kmers must be sorted when calling get_kmer_group_counts")
        return self._group_hist(kmer_len, kmer_filter_func, min_group_size, max_group_size, max_counts_bin)

    def _group_hist(self, kmer_len, kmer_filter_func, min_group_size, max_group_size, max_counts_bin):
        if max_counts_bin <= 0:
            raise ValueError(f"max_counts_bin ({max_counts_bin}) must be >= 1")
        _check_group_args(min_group_size, max_group_size, 1)
        self._sync_device()
        if self._engine.n == 0:
            return np.zeros(max_counts_bin + 1, dtype=np.int64), 0
        filt = self._filter_spec(kmer_filter_func)
        try:
            return self._engine.group_hist(self._is_sorted, kmer_len, filt, min_group_size, max_group_size,
                                           max_counts_bin)
        except _native.FilterRaised as e:
            raise _filter_error(e.ferr, e.sba_idx, kmer_filter_func) from None

    def get_unique_kmers(self) -> tuple:
        """(first sorted index, multiplicity) of every distinct k-mer at the sort length -- the
        unique/count output of the device pipeline (no reference counterpart beyond the groups)."""
        if not self._is_sorted:
            raise AssertionError("The kmers must be sorted when calling get_unique_kmers")
        self._sync_device()
        return self._engine.unique_counts()

    def get_encoded_kmers(self) -> np.ndarray:
        """Encoded keys of the sorted k-mers, one row per k-mer."""
        if not self._is_sorted:
            raise AssertionError("The kmers must be sorted when calling get_encoded_kmers")
        return self._engine.copy_keys()

    def generate_get_kmer_info_func(self, one_based_seq_index: bool) -> Callable:
        """Location-rich info per yielded k-mer (kmers.py:1180-1264)."""
        get_record_info = self.seq_coll.generate_get_record_info_from_sba_index_func(one_based_seq_index)

        def get_kmer_info(kmer_num, kmer_sba_start_indices, sba, kmer_len, group_size_yielded, group_size_total):
            if kmer_num < 0:
                raise ValueError(f"kmer_num ({kmer_num}) cannot be less than zero")
            if kmer_num >= len(kmer_sba_start_indices):
                raise ValueError(
                    f"kmer_num ({kmer_num}) is out of bounds (num kmers = {len(kmer_sba_start_indices)})"
                )
            sba_idx = int(kmer_sba_start_indices[kmer_num])
            _, _, seg_end, seq_strand, seq_chrom, seq_start_idx = get_record_info(sba_idx)
            if kmer_len is None:
                kmer_len = seg_end - sba_idx + 1
            elif sba_idx + kmer_len - 1 > seg_end:
                raise ValueError(
                    f"kmer_len ({kmer_len}) for kmer_num ({kmer_num}) extends beyond the end of the segment"
                )
            return (kmer_num, seq_strand, seq_chrom, seq_start_idx, kmer_len, group_size_yielded, group_size_total)

        return get_kmer_info

    # ---- equality / persistence (kmers.py:1266-1531) -----------------------------------------
    def __ne__(self, other):
        return not self.__eq__(other)

    def __eq__(self, other):
        if self.min_kmer_len != other.min_kmer_len:
            return False
        if (self.max_kmer_len is None) != (other.max_kmer_len is None) or self.max_kmer_len != other.max_kmer_len:
            return False
        for attr in ("kmer_source_strand", "track_strands_separately", "_is_initialized", "_is_set", "_is_sorted"):
            if getattr(self, attr) != getattr(other, attr):
                return False
        a, b = self.kmer_sba_start_indices, other.kmer_sba_start_indices
        if (a is None) != (b is None):
            return False
        if a is not None and not np.array_equal(a, b):
            return False
        if getattr(self, "seq_coll", None) != getattr(other, "seq_coll", None):
            return False
        return True

    def save(self, save_file_path: Path, include_sequence_collection: bool = False, format: str = "hdf5",
             mode: str = "w") -> None:
        if format == "hdf5":
            self._save_hdf5(save_file_path, include_sequence_collection, mode=mode)
        elif format == "shelve":
            self._save_shelve(save_file_path, include_sequence_collection)
        else:
            raise ValueError(f"format ({format}) not recognized")

    def load(self, load_file_path: Path, seq_coll: Union[SequenceCollection, None] = None,
             format: str = "hdf5") -> None:
        if format == "hdf5":
            self._load_hdf5(load_file_path, seq_coll)
        elif format == "shelve":
            self._load_shelve(load_file_path, seq_coll)
        else:
            raise ValueError(f"format ({format}) not recognized")

    def _save_hdf5(self, save_file_path, include_sequence_collection=False, mode="w"):
        import h5py

        with h5py.File(save_file_path, mode) as f:
            g = f.create_group("kmers")
            g["min_kmer_len"] = self.min_kmer_len
            g["max_kmer_len"] = 0 if self.max_kmer_len is None else self.max_kmer_len
            g["kmer_source_strand"] = self.kmer_source_strand
            g["track_strands_separately"] = self.track_strands_separately
            g["_is_initialized"] = self._is_initialized
            g["_is_set"] = self._is_set
            # a canonical order is not the reference's sort order: the file says "not sorted" to the
            # reference's loader (kmers.py:939-960, 1435-1472), which then treats the object as
            # unsorted, and keeps the canonical state in keys of its own, which only this build reads
            g["_is_sorted"] = False if self._canonical else self._is_sorted
            s = self.kmer_sba_start_indices
            g["kmer_sba_start_indices"] = np.array([], dtype=np.uint32) if s is None else s
            if self._canonical:
                g["_canonical"] = True
                g["_canonical_sorted"] = bool(self._is_sorted)
        if include_sequence_collection:
            self.seq_coll.save(save_file_path, mode="a", format="hdf5")

    def _restore(self, starts, seq_coll, canonical=False):
        self.seq_coll = seq_coll
        self._engine = None
        if starts is not None and seq_coll is not None and seq_coll.forward_sba is not None:
            self.kmer_sba_start_indices = np.asarray(starts, dtype=np.uint32)
        else:
            self._host_starts = starts
            self._host_valid = True
            self._device_stale = starts is not None
        # a canonical sort saved by this build (the reference has no canonical order); any other
        # file restores a forward order, whatever this object held before
        self._canonical = bool(canonical)

    def _load_hdf5(self, load_file_path, seq_coll=None):
        import h5py

        with h5py.File(load_file_path, "r") as f:
            g = f["kmers"]
            self.min_kmer_len = g["min_kmer_len"][()]
            mk = g["max_kmer_len"][()]
            self.max_kmer_len = None if mk == 0 else mk
            self.kmer_source_strand = g["kmer_source_strand"][()].decode("utf-8")
            self.track_strands_separately = g["track_strands_separately"][()]
            self._is_initialized = g["_is_initialized"][()]
            self._is_set = g["_is_set"][()]
            self._is_sorted = g["_is_sorted"][()]
            s = g["kmer_sba_start_indices"][:]
            starts = None if s.shape == (0,) else s
            canonical = bool(g["_canonical"][()]) if "_canonical" in g else False
            if canonical:
                # a canonical file written before the key existed: keep the stored flag
                if "_canonical_sorted" in g:
                    self._is_sorted = bool(g["_canonical_sorted"][()])
        if seq_coll is None:
            seq_coll = SequenceCollection()
            seq_coll.load(load_file_path, format="hdf5")
        self._restore(starts, seq_coll, canonical)

    def _save_shelve(self, save_file_path, include_sequence_collection=False):
        with shelve.open(str(save_file_path)) as db:
            for k in ("min_kmer_len", "max_kmer_len", "kmer_source_strand", "track_strands_separately",
                      "_is_initialized", "_is_set", "_is_sorted"):
                db[k] = getattr(self, k)
            db["kmer_sba_start_indices"] = self.kmer_sba_start_indices
            if self._canonical:  # as _save_hdf5: "not sorted" for the reference, canonical state apart
                db["_is_sorted"] = False
                db["_canonical"] = True
                db["_canonical_sorted"] = bool(self._is_sorted)
        if include_sequence_collection:
            self.seq_coll.save(save_file_path, format="shelve")

    def _load_shelve(self, load_file_path, seq_coll=None):
        with shelve.open(str(load_file_path)) as db:
            for k in ("min_kmer_len", "max_kmer_len", "kmer_source_strand", "track_strands_separately",
                      "_is_initialized", "_is_set", "_is_sorted"):
                setattr(self, k, db[k])
            starts = db["kmer_sba_start_indices"]
            canonical = bool(db.get("_canonical", False))
            if canonical:
                self._is_sorted = bool(db.get("_canonical_sorted", self._is_sorted))
        if seq_coll is None:
            seq_coll = SequenceCollection()
            seq_coll.load(load_file_path, format="shelve")
        self._restore(starts, seq_coll, canonical)

    # ---- readback (kmers.py:1533-1622) -------------------------------------------------------
    def _start_at(self, kmer_num: int) -> int:
        if self._host_valid and self._host_starts is not None:
            return int(self._host_starts[kmer_num])
        return int(self._engine.start_range(kmer_num, 1)[0])

    def get_kmer_str_no_checks(self, kmer_num: int, kmer_strand: str, kmer_len: int) -> str:
        if kmer_strand == "+":
            sba = self.seq_coll.forward_sba
            start = self._start_at(kmer_num)
        elif kmer_strand == "-":
            raise NotImplementedError("Only implemented for kmer_strand='+'")
        else:
            raise ValueError(f"kmer_strand ({kmer_strand}) not recognized")
        return bytes(sba[start : start + kmer_len]).decode("utf-8")

    def get_kmer_str(self, kmer_num: int, kmer_len: Union[int, None] = None) -> str:
        self._check_forward()
        if kmer_num < 0:
            raise ValueError(f"kmer_num ({kmer_num}) cannot be less than zero")
        if kmer_num >= len(self):
            raise ValueError(f"kmer_num ({kmer_num}) is out of bounds (num kmers = {len(self)})")
        if kmer_len is not None and kmer_len < self.min_kmer_len:
            raise ValueError(f"kmer_len ({kmer_len}) is less than min_kmer_len ({self.min_kmer_len})")
        if self.max_kmer_len is not None and kmer_len > self.max_kmer_len:  # TypeError for None, as kmers.py:1599
            raise ValueError(f"kmer_len ({kmer_len}) is greater than max_kmer_len ({self.max_kmer_len})")
        start = self._start_at(kmer_num)
        seg = self.seq_coll.get_segment_num_from_sba_index(start)
        _, seg_end = self.seq_coll.get_sba_start_end_indices_for_segment(seg)
        if kmer_len is None:
            largest = seg_end - start + 1
            kmer_len = largest if self.max_kmer_len is None else min(self.max_kmer_len, largest)
        if start + kmer_len - 1 > seg_end:
            raise ValueError(f"kmer_len ({kmer_len}) for kmer_num ({kmer_num}) extends beyond the end of the segment")
        return bytes(self.seq_coll.forward_sba[start : start + kmer_len]).decode("utf-8")

    # ---- sort (kmers.py:1624-1731) -----------------------------------------------------------
    def sort(self, *, canonical: bool = False, order: str = "stable"):
        """Sort the start indices by k-mer on the GPU (in place from the caller's point of view).

        Tie order (``order="stable"``, the default): equal k-mers come back in ascending start
        order -- the reference's ``get_is_less_than_func(break_ties=True)`` order
        (kmers.py:1710-1711).  The reference's own ``sort()`` uses ``break_ties=False`` and leaves
        equal k-mers in whatever order numba's quicksort produces (kmers.py:1624-1652); no parallel
        sort reproduces that.  ``order="reference"`` gives exactly that order: the device sorts,
        then numba's quicksort runs on the host over the original start order, comparing the
        device's group ranks (libgkm GK_SORT_QUICKSORT_ORDER; host-bound, 8 B of host memory per k-mer, not
        with canonical=True).  Sorted k-mers,
        encoded keys, group sizes, counts, histograms and the ``(kmer_num, group_size_yielded,
        group_size_total)`` tuples of ``get_kmers`` are identical either way, because ties only
        permute the members of a group inside the group's index range.  What can differ is WHICH
        members a tie group reports: the start (and so the location) behind a given ``kmer_num``
        inside a group, i.e. the members ``yield_first_n`` picks and the locations of
        ``kmer_info_to_yield="full"``.  Here they are the group's smallest start indices.

        canonical=True (this build's extension; the reference has no canonical k-mers,
        kmers.py:689-696): order by min(k-mer, reverse complement) with the reference's IUPAC
        complement (sequence_collection.py:402-433).  Needs min_kmer_len == max_kmer_len; groups,
        counts and encoded keys then refer to canonical k-mers (at kmer_len == max_kmer_len), and
        get_canonical_strands() tells which strand each sorted k-mer's canonical form came from.
        """
        self._check_forward()
        if order not in ("stable", "reference"):
            raise ValueError(f"order must be 'stable' or 'reference' (order = {order!r})")
        if canonical and order == "reference":
            raise ValueError("order='reference' is the reference's forward-strand quicksort order; the reference "
                             "has no canonical k-mers")
        if canonical and (self.max_kmer_len is None or self.max_kmer_len != self.min_kmer_len):
            raise ValueError(f"canonical k-mers need min_kmer_len == max_kmer_len (min_kmer_len = "
                             f"{self.min_kmer_len}, max_kmer_len = {self.max_kmer_len})")
        self._sync_device()
        try:
            self._engine.sort(self.max_kmer_len, canonical=canonical, quicksort_order=order == "reference")
        except _native.GkError as e:
            if e.code == _native.GK_E_NO_BASES:
                raise AssertionError(
                    f"kmers compared were less than min_kmer_len ({self.min_kmer_len}).  Was "
                    "kmer_sba_start_indices initialized correctly?"
                ) from None
            raise
        self._after_device_reorder()
        self._is_sorted = True
        self._canonical = canonical

    def get_canonical_strands(self) -> np.ndarray:
        """uint8 per sorted k-mer after sort(canonical=True): 1 if the canonical form is the k-mer's
        reverse complement (strictly smaller), 0 if it is the k-mer itself (or a palindrome)."""
        if not (self._is_sorted and self._canonical):
            raise AssertionError("get_canonical_strands needs sort(canonical=True)")
        return self._engine.copy_strands()

    def get_is_less_than_func(self, validate_kmers: bool = True, break_ties: bool = False) -> Callable:
        """Scalar is_less_than(a, b) of the reference (kmers.py:1654-1731), host-side, for callers
        that compare individual k-mers; Kmers.sort() does not use it."""
        self._check_forward()
        sba = self.seq_coll.forward_sba
        min_kmer_len, max_kmer_len = self.min_kmer_len, self.max_kmer_len

        def is_less_than(a: int, b: int) -> bool:
            comparison, last = compare_sba_kmers_lexicographically(sba, sba, a, b, max_kmer_len=max_kmer_len)
            if comparison < 0:
                lt = True
            elif comparison > 0:
                lt = False
            else:
                lt = (a < b) if break_ties else False
            if validate_kmers:
                nb = min_kmer_len - (last + 1)
                if not kmer_has_required_len(sba, a + last + 1, nb) or not kmer_has_required_len(sba, b + last + 1, nb):
                    raise AssertionError(
                        f"kmers compared were less than min_kmer_len ({min_kmer_len}).  Was "
                        "kmer_sba_start_indices initialized correctly?"
                    )
            return lt

        return is_less_than

    def to_csv(self, kmer_len, output_file_path, fields=["kmer"]):
        pass
