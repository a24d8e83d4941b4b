"""Device contract checks added in round 3 (all through libgkm.so's C ABI):

* the reference's default ``sort()`` tie order vs this build's ``break_ties=True`` order: every
  order-independent output -- keys, group sizes, counts, histograms, and the ``(kmer_num,
  size_yielded, size_total)`` tuples of ``get_kmers`` -- equals the reference's DEFAULT-order
  results (``results_default_order`` in tests/golden/manifest.json, produced by running the
  reference); only the starts inside tie groups differ (kmers.py:1624-1731);
* custom ``kmer_comparison_func`` callables in the module-level group helpers
  (kmers.py:285-303, 454-648): groups decided on the host, counted on the device -- checked against
  the built-in comparator and against a plain restatement of the reference generator;
* determinism: the same input sorted twice in fresh engines gives byte-identical starts, keys and
  unique counts.
"""

import numpy as np
import pytest

from conftest import load_case, load_manifest
from genome_kmers import _native
from genome_kmers import kmers as gk
from genome_kmers import synthetic
from oracle import oracle
from test_gpu_parity import make, run_query

pytestmark = pytest.mark.gpu

CASES = load_manifest()
TIE_CASES = [c for c in CASES if c["ties_differ"]]


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert _native.device_count() > 0, "gpu tests need a visible MI355X"


# ---------------------------------------------------------------------------------------------
# default tie order: the difference is confined to the members of tie groups
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("case", TIE_CASES, ids=lambda c: c["name"])
def test_default_order_differs_only_inside_tie_groups(case):
    km, a = make(case)
    km.sort()
    starts = km.kmer_sba_start_indices
    # the same multiset of starts, and every difference lies inside a group of equal k-mers
    assert sorted(starts.tolist()) == sorted(a["starts_default"].tolist())
    diff = np.flatnonzero(starts != a["starts_default"])
    assert len(diff) > 0, "the case has tie groups whose quicksort order differs"
    if case["max_kmer_len"] is not None:
        sba, mk = a["sba"], case["max_kmer_len"]
        for i in diff.tolist():
            assert bytes(sba[starts[i]:starts[i] + mk]).split(b"$")[0] == \
                bytes(sba[a["starts_default"][i]:a["starts_default"][i] + mk]).split(b"$")[0]
        # encoded keys: the reference's default order gives the same key sequence
        words, bits, _ = km._engine.key_layout()
        if bits:
            spec = oracle.key_spec(km._engine.is_acgt(), case["min_kmer_len"], case["max_kmer_len"])
            np.testing.assert_array_equal(km.get_encoded_kmers(),
                                          oracle.encode_keys(a["sba"], a["starts_default"], *spec))
    # group queries whose answer does not name a member's location: identical to the reference's
    # default-order answers (kmer_num indexes the sorted order; groups occupy the same ranges)
    checked = 0
    for q, want in zip(case["queries"], case["results_default_order"]):
        if q.get("info", "minimum") == "full":
            continue
        assert run_query(km, q) == want, q
        checked += 1
    assert checked > 0


# ---------------------------------------------------------------------------------------------
# custom comparison callbacks
# ---------------------------------------------------------------------------------------------
def reference_generator(sba, kmer_len, starts, cmp, filt, min_g=1, max_g=None, first_n=None):
    """Plain restatement of kmer_info_by_group_generator (kmers.py:523-648) with
    get_kmer_info_minimal: the test's ground truth for arbitrary comparators."""
    out, members, size, prev = [], [], 0, None

    def flush():
        if size >= min_g and (max_g is None or size <= max_g):
            out.extend((k, len(members), size) for k in members)

    for num, s in enumerate(starts.tolist()):
        if not filt(sba, "forward", s):
            continue
        same = True if prev is None else cmp(sba, sba, prev, s)[0] == 0
        prev = s
        if same:
            size += 1
            if first_n is None or len(members) < first_n:
                members.append(num)
        else:
            flush()
            size, members = 1, [num]
    flush()
    return out


def _sorted_case(name):
    case = next(c for c in CASES if c["name"] == name)
    a = load_case(name)
    return case, a["sba"], a["starts_stable"]


@pytest.mark.parametrize("name", ["c1_seed42_10kb_k5", "seq2_min3_max3"])
def test_custom_comparator_equals_builtin(name):
    """A user lambda doing what get_compare_sba_kmers_func(k) does gives the built-in answers."""
    case, sba, starts = _sorted_case(name)
    k = case["max_kmer_len"]

    def my_cmp(sba_a, sba_b, ia, ib):  # a plain Python callable, not the library's comparator
        return gk.compare_sba_kmers_lexicographically(sba_a, sba_b, ia, ib, max_kmer_len=k)

    builtin = gk.get_compare_sba_kmers_func(k)
    for filt in (gk.kmer_filter_keep_all, gk.gen_kmer_homopolymer_filter_func(2, k)):
        for mg, xg, fn in ((1, None, None), (2, None, 1), (1, 3, 2)):
            h1, t1 = gk.get_kmer_group_size_hist(sba, "forward", k, starts, my_cmp, filt, mg, xg, 64)
            h2, t2 = gk.get_kmer_group_size_hist(sba, "forward", k, starts, builtin, filt, mg, xg, 64)
            np.testing.assert_array_equal(h1, h2)
            assert t1 == t2
            g1 = list(gk.kmer_info_by_group_generator(sba, "forward", k, starts, my_cmp, filt,
                                                      gk.get_kmer_info_minimal, mg, xg, fn))
            g2 = list(gk.kmer_info_by_group_generator(sba, "forward", k, starts, builtin, filt,
                                                      gk.get_kmer_info_minimal, mg, xg, fn))
            assert g1 == g2
            assert g1 == reference_generator(sba, k, starts, my_cmp, filt, mg, xg, fn)


def test_custom_comparator_own_semantics():
    """A comparator no built-in reproduces (the first two bases and the parity of the third byte)
    with a custom filter: host-decided groups, device-counted, vs the reference generator."""
    case, sba, starts = _sorted_case("c1_seed42_10kb_k5")

    def two_bases(sba_a, sba_b, ia, ib):
        a, b = bytes(sba_a[ia:ia + 2]), bytes(sba_b[ib:ib + 2])
        pa, pb = int(sba_a[ia + 2]) & 1, int(sba_b[ib + 2]) & 1
        return (0 if (a, pa) == (b, pb) else (-1 if (a, pa) < (b, pb) else 1)), 2

    def no_t_start(sba_, strand, idx):
        return sba_[idx] != ord("T")

    for mg, xg, fn in ((1, None, None), (3, None, 2), (2, 40, 1)):
        want = reference_generator(sba, 5, starts, two_bases, no_t_start, mg, xg, fn)
        got = list(gk.kmer_info_by_group_generator(sba, "forward", 5, starts, two_bases, no_t_start,
                                                   gk.get_kmer_info_minimal, mg, xg, fn))
        assert got == want
        # the histogram: one yield per group (kmers.py:497-518)
        groups = reference_generator(sba, 5, starts, two_bases, no_t_start, mg, xg, 1)
        wh = np.zeros(51, dtype=np.int64)
        for g in groups:
            wh[min(g[2], 50)] += 1
        h, t = gk.get_kmer_group_size_hist(sba, "forward", 5, starts, two_bases, no_t_start, mg, xg, 50)
        np.testing.assert_array_equal(h, wh)
        assert t == sum(g[2] for g in groups)


def test_custom_comparator_filter_raise_matches_reference():
    """A built-in filter that raises while a custom comparator groups: the reference's error."""
    case, sba, starts = _sorted_case("seq2_min3_max3")

    def my_cmp(sba_a, sba_b, ia, ib):
        return gk.compare_sba_kmers_lexicographically(sba_a, sba_b, ia, ib, max_kmer_len=3)

    filt = gk.gen_no_ambiguous_bases_filter(9)  # runs past a '$' for some starts
    with pytest.raises(ValueError) as e_ref:
        reference_generator(sba, 3, starts, my_cmp, filt)
    with pytest.raises(ValueError) as e_dev:
        list(gk.kmer_info_by_group_generator(sba, "forward", 3, starts, my_cmp, filt, gk.get_kmer_info_minimal))
    assert str(e_dev.value) == str(e_ref.value)


# ---------------------------------------------------------------------------------------------
# determinism: two fresh engines, byte-identical products
# ---------------------------------------------------------------------------------------------
def _product(sba, seg, k, canonical=False):
    eng = _native.Engine()
    eng.set_sequence(sba, seg)
    eng.enumerate(k)
    eng.sort(k, canonical=canonical)
    starts = np.empty(eng.n, dtype=np.uint32)
    eng.copy_starts(starts)
    keys = eng.copy_keys()
    ustart, ucount = eng.unique_counts()
    return starts, keys, ustart, ucount


@pytest.mark.parametrize("which", ["c2_k31", "iupac_k63", "iupac_k63_canonical"])
def test_sort_is_deterministic(which):
    if which == "c2_k31":
        sba, seg = synthetic.c2_surrogate()
        k, canonical = 31, False
    else:
        rng = np.random.default_rng(5)
        s = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, 1_500_000)].copy()
        at = rng.integers(0, len(s), 3000)
        s[at] = np.frombuffer(b"NRYKMSWBDHV", dtype=np.uint8)[rng.integers(0, 11, len(at))]
        s[200_000:260_000] = ord("N")
        rep = s[500_000:503_000].copy()
        for p in rng.integers(0, len(s) - 3000, 12):
            s[p:p + 3000] = rep
        sba = np.concatenate([s[:900_000], [36], s[900_000:]]).astype(np.uint8)
        seg = np.array([0, 900_001], dtype=np.uint32)
        k, canonical = 63, which.endswith("canonical")
    a = _product(sba, seg, k, canonical)
    b = _product(sba, seg, k, canonical)
    for x, y in zip(a, b):
        assert x.dtype == y.dtype and x.shape == y.shape
        assert x.tobytes() == y.tobytes()
    # and the product is the oracle's order (stable ties)
    if not canonical:
        want = oracle.quicksort(sba, oracle.enumerate_starts(sba, seg, k), k, k, break_ties=True)
        np.testing.assert_array_equal(a[0], want)
