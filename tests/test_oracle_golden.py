"""Pin the CPU oracle against golden vectors produced by the reference itself (CPU only).

The golden vectors (tests/golden/*.npz + manifest.json) come from running mrperkett/genome-kmers
v1.0.1 with tests/golden/make_golden.py.  If the oracle reproduces them, it is trusted as the
checker for the device path at sizes the reference cannot reach.
"""

import numpy as np
import pytest

from conftest import load_case, load_manifest
from oracle import oracle

CASES = load_manifest()
CASE_IDS = [c["name"] for c in CASES]


@pytest.mark.parametrize("case", CASES, ids=CASE_IDS)
def test_enumerate_matches_reference(case):
    a = load_case(case["name"])
    got = oracle.enumerate_starts(a["sba"], a["seg_starts"], case["min_kmer_len"])
    np.testing.assert_array_equal(got, a["starts_unsorted"])


@pytest.mark.parametrize("case", CASES, ids=CASE_IDS)
def test_quicksort_default_order_matches_reference(case):
    """numba-quicksort restatement reproduces the reference's default tie order bit-exactly."""
    a = load_case(case["name"])
    got = oracle.quicksort(a["sba"], a["starts_unsorted"], case["min_kmer_len"], case["max_kmer_len"])
    np.testing.assert_array_equal(got, a["starts_default"])


@pytest.mark.parametrize("case", CASES, ids=CASE_IDS)
def test_quicksort_break_ties_matches_reference(case):
    a = load_case(case["name"])
    got = oracle.quicksort(a["sba"], a["starts_unsorted"], case["min_kmer_len"], case["max_kmer_len"],
                           break_ties=True)
    np.testing.assert_array_equal(got, a["starts_stable"])


def _run_query(sba, starts, q):
    filt = oracle.filter_params(q["filter"])
    try:
        if q["op"] == "group_counts":
            h, t = oracle.group_scan(sba, starts, q["kmer_len"], filt, q["min_group_size"], q["max_group_size"],
                                     max_counts_bin=q["max_counts_bin"])
            return {"hist": h.tolist(), "total": t}
        if q["op"] == "count":
            _, t = oracle.group_scan(sba, starts, q["kmer_len"], filt, q["min_group_size"], q["max_group_size"],
                                     max_counts_bin=1000000)
            return {"total": t}
        ys = oracle.group_scan(sba, starts, q["kmer_len"], filt, q["min_group_size"], q["max_group_size"],
                               yield_first_n=q.get("yield_first_n"))
        return {"yields": [list(y) for y in ys]}
    except oracle.OracleError as e:
        return {"error": e.kind, "idx": e.idx}


def _golden_yields(res, info):
    if info == "full":  # (kmer_num, strand, chrom, seq_idx, kmer_len, yielded, total)
        return [[r[0], r[5], r[6]] for r in res["kmers"]]
    return [list(r) for r in res["kmers"]]


@pytest.mark.parametrize("order", ["default", "stable"])
@pytest.mark.parametrize("case", CASES, ids=CASE_IDS)
def test_group_queries_match_reference(case, order):
    a = load_case(case["name"])
    starts = a[f"starts_{order}"]
    results = case[f"results_{order}_order"]
    for q, want in zip(case["queries"], results):
        got = _run_query(a["sba"], starts, q)
        if "error" in want:
            assert "error" in got, (q, got)
            continue
        assert "error" not in got, (q, got)
        if q["op"] == "group_counts":
            assert got["hist"] == want["hist"], q
            assert got["total"] == want["total"], q
        elif q["op"] == "count":
            assert got["total"] == want["total"], q
        else:
            assert got["yields"] == _golden_yields(want, q.get("info", "minimum")), q


def test_golden_covers_ties_and_modes():
    """The fixture set exercises what the device must get right."""
    assert any(c["ties_differ"] for c in CASES)
    assert any(c["max_kmer_len"] is None for c in CASES)
    assert any(c["max_kmer_len"] not in (None, c["min_kmer_len"]) for c in CASES)
    assert any("error" in r for c in CASES for r in c["results_default_order"])


def test_docs_example_suffix_order():
    """docs/resources/kmer-sba-diagram.png: seq_list_2, min_kmer_len=3, max None."""
    a = load_case("seq2_min3_maxNone")
    assert a["starts_default"].tolist() == [4, 31, 0, 13, 20, 5, 27, 19, 32, 33, 34, 2, 15, 3, 30, 12, 26, 18, 11,
                                            24, 7, 1, 14, 29, 25, 17, 6, 28, 16]


# ---------------------------------------------------------------------------------------------
# the key encoding is order-isomorphic to the reference comparator
# ---------------------------------------------------------------------------------------------
def _random_sba(rng, n, alphabet):
    s = rng.choice(np.frombuffer(alphabet, dtype=np.uint8), n)
    cuts = np.arange(1, 7) * (n // 7) + rng.integers(-5, 5, 6)
    s[cuts] = 36
    return s.astype(np.uint8)


@pytest.mark.parametrize("alphabet,is_acgt", [(b"ACGT", True), (b"ACGTNRYKM", False), (b"AAAC", True)])
@pytest.mark.parametrize("min_k,max_k", [(5, 5), (31, 31), (3, 12), (1, 40), (32, 32), (20, 64)])
def test_key_order_isomorphic_to_comparator(alphabet, is_acgt, min_k, max_k):
    rng = np.random.default_rng(min_k * 100 + max_k + len(alphabet))
    sba = _random_sba(rng, 600, alphabet)
    seg = np.concatenate([[0], np.flatnonzero(sba == 36) + 1]).astype(np.uint32)
    if min(np.diff(np.append(seg, len(sba) + 1))) - 1 < min_k:
        pytest.skip("segment shorter than min_k")
    starts = oracle.enumerate_starts(sba, seg, min_k)
    spec = oracle.key_spec(is_acgt, min_k, max_k)
    keys = oracle.encode_keys(sba, starts, *spec)
    as_int = [int.from_bytes(b"".join(int(w).to_bytes(8, "big") for w in row), "big") for row in keys]
    pairs = rng.integers(0, len(starts), size=(3000, 2))
    for i, j in pairs:
        c, _ = oracle.compare(sba, int(starts[i]), int(starts[j]), max_k)
        d = (as_int[i] > as_int[j]) - (as_int[i] < as_int[j])
        assert c == d, (int(starts[i]), int(starts[j]))


def test_complement_mapping_pinned_to_reference():
    """The canonical extension's complement = the reference's (tests/golden/make_complement.py)."""
    z = load_case("complement")
    np.testing.assert_array_equal(oracle.COMPLEMENT_LUT, z["complement_lut"])
    np.testing.assert_array_equal(oracle.reverse_complement(z["sba"]), z["rc_sba"])
    np.testing.assert_array_equal(oracle.reverse_complement(z["sba"]), z["both_sba"])


def test_canonical_oracle_small_cases():
    sba = np.frombuffer(b"ACGTTGCAAC$GGCC", dtype=np.uint8)
    starts = np.array([0, 1, 2, 3, 4, 5, 6, 11], dtype=np.uint32)
    canon, is_rc = oracle.canonical_windows(sba, starts, 4)
    assert [bytes(c) for c in canon] == [b"ACGT", b"AACG", b"CAAC", b"GCAA", b"TGCA", b"GCAA", b"CAAC", b"GGCC"]
    assert is_rc.tolist() == [False, True, True, True, False, False, False, False]
    srt = oracle.canonical_sort(sba, starts, 4)
    assert srt.tolist() == [1, 0, 2, 6, 3, 5, 11, 4]
    hist, total = oracle.canonical_group_hist(sba, srt, 4, 5)
    assert hist.tolist() == [0, 4, 2, 0, 0, 0] and total == 8
    # canonical keys are the forward keys of the canonical bytes
    keys = oracle.canonical_keys(sba, srt, 4, 2)
    assert np.all(keys[1:, 0] >= keys[:-1, 0])
