"""Device parity: the drop-in Kmers API (libgkm.so through its C ABI) vs the reference's golden
vectors and the CPU oracle.  Bit-exact for every integer output.

Contract: start indices equal the reference's break_ties=True order (equal
k-mers by ascending start index); k-mer order, keys, group histograms, counts and generator
yields equal the reference on that order.
"""

import numpy as np
import pytest

from conftest import load_case, load_manifest, seq_list_of
from genome_kmers import _native
from genome_kmers import kmers as gk
from genome_kmers.sequence_collection import SequenceCollection
from oracle import oracle

pytestmark = pytest.mark.gpu

CASES = load_manifest()
CASE_IDS = [c["name"] for c in CASES]


def make(case):
    a = load_case(case["name"])
    sc = SequenceCollection(sequence_list=seq_list_of(case, a), strands_to_load="forward")
    np.testing.assert_array_equal(sc.forward_sba, a["sba"])
    np.testing.assert_array_equal(sc._forward_sba_seg_starts, a["seg_starts"])
    km = gk.Kmers(sc, min_kmer_len=case["min_kmer_len"], max_kmer_len=case["max_kmer_len"])
    return km, a


def filter_of(spec):
    k = spec["kind"]
    if k == "keep_all":
        return gk.kmer_filter_keep_all
    if k == "length":
        return gk.gen_kmer_length_filter_func(spec["min_kmer_len"])
    if k == "homopolymer":
        return gk.gen_kmer_homopolymer_filter_func(spec["max_homopolymer_size"], spec["kmer_len"])
    if k == "gc":
        return gk.gen_kmer_gc_content_filter_func(spec["min_gc"], spec["max_gc"], spec["kmer_len"])
    if k == "no_ambiguous":
        return gk.gen_no_ambiguous_bases_filter(spec["kmer_len"])
    if k == "crispr_ngg":
        return gk.crispr_ngg_pam_filter
    raise ValueError(k)


def run_query(km, q):
    filt = filter_of(q["filter"])
    try:
        if q["op"] == "group_counts":
            h, t = km.get_kmer_group_counts(q["kmer_len"], filt, q["min_group_size"], q["max_group_size"],
                                            q["max_counts_bin"])
            return {"hist": h.tolist(), "total": int(t)}
        if q["op"] == "count":
            return {"total": int(km.get_kmer_count(q["kmer_len"], filt, q["min_group_size"], q["max_group_size"]))}
        out = list(km.get_kmers(q["kmer_len"], kmer_filter_func=filt, kmer_info_to_yield=q.get("info", "minimum"),
                                min_group_size=q["min_group_size"], max_group_size=q["max_group_size"],
                                yield_first_n=q.get("yield_first_n"), one_based_seq_index=q.get("one_based", False)))
        return {"kmers": [list(t) for t in out]}
    except (ValueError, AssertionError) as e:
        return {"error": type(e).__name__, "message": str(e)}


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert _native.device_count() > 0, "gpu tests need a visible MI355X"


# ---------------------------------------------------------------------------------------------
# golden vectors (produced by the reference itself)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("case", CASES, ids=CASE_IDS)
def test_enumerate_golden(case):
    km, a = make(case)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, a["starts_unsorted"])
    assert len(km) == case["num_kmers"]


@pytest.mark.parametrize("case", CASES, ids=CASE_IDS)
def test_sort_golden(case):
    km, a = make(case)
    km.sort()
    np.testing.assert_array_equal(km.kmer_sba_start_indices, a["starts_stable"])
    # same k-mer sequence as the reference's default order (ties only permute equal k-mers)
    if case["max_kmer_len"] is not None:
        sba, mk = a["sba"], case["max_kmer_len"]
        got = [bytes(sba[s:s + mk]).split(b"$")[0] for s in km.kmer_sba_start_indices.tolist()]
        ref = [bytes(sba[s:s + mk]).split(b"$")[0] for s in a["starts_default"].tolist()]
        assert got == ref


@pytest.mark.parametrize("case", [c for c in CASES if c["max_kmer_len"] is not None], ids=lambda c: c["name"])
def test_encoded_keys_golden(case):
    km, a = make(case)
    km.sort()
    words, bits, symbols = km._engine.key_layout()
    if bits == 0:
        pytest.skip("long bound sorted by prefix doubling: keys are ranks")
    acgt = km._engine.is_acgt()
    spec = oracle.key_spec(acgt, case["min_kmer_len"], case["max_kmer_len"])
    assert (words, bits, symbols) == (spec[3], spec[0], spec[1])
    want = oracle.encode_keys(a["sba"], a["starts_stable"], *spec)
    np.testing.assert_array_equal(km.get_encoded_kmers(), want)


@pytest.mark.parametrize("case", CASES, ids=CASE_IDS)
def test_group_queries_golden(case):
    km, _ = make(case)
    km.sort()
    for q, want in zip(case["queries"], case["results_stable_order"]):
        got = run_query(km, q)
        assert got == want, q


@pytest.mark.parametrize("case", [c for c in CASES if not c["ties_differ"]], ids=lambda c: c["name"])
def test_default_order_equals_when_no_ties(case):
    km, a = make(case)
    km.sort()
    np.testing.assert_array_equal(km.kmer_sba_start_indices, a["starts_default"])
    for q, want in zip(case["queries"], case["results_default_order"]):
        assert run_query(km, q) == want, q


def test_unsorted_queries_every_kmer_its_own_group():
    case = next(c for c in CASES if c["name"] == "c1_seed42_10kb_k5")
    km, a = make(case)
    assert km.get_kmer_count(5) == len(a["starts_unsorted"])
    got = list(km.get_kmers(5))
    assert got == [(i, 1, 1) for i in range(len(a["starts_unsorted"]))]
    with pytest.raises(AssertionError, match="must be sorted"):
        km.get_kmer_group_counts(5)


def test_get_kmer_str_after_sort():
    case = next(c for c in CASES if c["name"] == "seq2_min3_maxNone")
    km, a = make(case)
    km.sort()
    sba = a["sba"]
    for i, s in enumerate(a["starts_stable"].tolist()):
        end = bytes(sba[s:]).split(b"$")[0]
        assert km.get_kmer_str(i) == end.decode()


# ---------------------------------------------------------------------------------------------
# oracle parity at larger sizes
# ---------------------------------------------------------------------------------------------
def random_genome(rng, lengths, alphabet=b"ACGT", repeat=None, copies=0):
    seqs = []
    for i, L in enumerate(lengths):
        s = rng.choice(np.frombuffer(alphabet, dtype=np.uint8), L).astype(np.uint8)
        if repeat is not None:
            for _ in range(copies):
                at = int(rng.integers(0, max(1, L - len(repeat))))
                s[at:at + len(repeat)] = repeat[: L - at]
        seqs.append((f"c{i}", s.tobytes().decode()))
    return seqs


def oracle_check(seqs, min_k, max_k, check_counts=True):
    sc = SequenceCollection(sequence_list=seqs)
    km = gk.Kmers(sc, min_kmer_len=min_k, max_kmer_len=max_k)
    unsorted = oracle.enumerate_starts(sc.forward_sba, sc._forward_sba_seg_starts, min_k)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, unsorted)
    km.sort()
    want = oracle.quicksort(sc.forward_sba, unsorted, min_k, max_k, break_ties=True)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)
    if check_counts:
        kl = max_k if max_k is not None else min_k
        h, t = km.get_kmer_group_counts(kl, max_counts_bin=64)
        oh, ot = oracle.group_scan(sc.forward_sba, want, kl, max_counts_bin=64)
        np.testing.assert_array_equal(h, oh)
        assert t == ot
    return km, sc, want


@pytest.mark.parametrize("seed", [1, 2])
def test_random_acgt_k31_vs_oracle(seed):
    rng = np.random.default_rng(seed)
    oracle_check(random_genome(rng, [300_000, 150_000, 31, 77_777]), 31, 31)


def test_repeats_and_ties_k31_vs_oracle():
    rng = np.random.default_rng(3)
    rep = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 5000).astype(np.uint8)
    oracle_check(random_genome(rng, [200_000, 120_000], repeat=rep, copies=7), 31, 31)


def test_homopolymer_genome_all_ties():
    seqs = [("a", "A" * 50_000), ("b", "A" * 20_000 + "C" * 20_000)]
    oracle_check(seqs, 21, 21)


# MSD depth: inputs whose buckets stay above the local limit (4096) for several global levels
# (the random cases above finish after L0 / L1), at every level digit width (GKM_LEVEL_BITS)
@pytest.mark.parametrize("level_bits", ["8", "8,7", "8,6", "8,7,8", "7,8,8", "6,8,8"])
def test_low_entropy_deep_levels_vs_oracle(level_bits, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_LEVEL_BITS", level_bits)
    rng = np.random.default_rng(11)
    # 1 bit per base: L0 leaves 16 buckets of ~150K, L1 ~10K each, L2 below the local limit
    oracle_check(random_genome(rng, [1_600_000, 800_000], alphabet=b"AC"), 31, 31)


@pytest.mark.parametrize("level_bits", ["8", "8,7,8", "7,8,8"])
def test_sparse_variation_all_levels_vs_oracle(level_bits, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_LEVEL_BITS", level_bits)
    rng = np.random.default_rng(12)
    # mostly 'A' with a random base every ~40: huge equal-prefix buckets down to the last key bit,
    # exhausted (all-equal) buckets far above the local limit, long runs of ties
    s = np.full(600_000, ord("A"), dtype=np.uint8)
    at = rng.integers(0, len(s), len(s) // 40)
    s[at] = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, len(at))]
    oracle_check([("a", s[:450_000].tobytes().decode()), ("b", s[450_000:].tobytes().decode())], 31, 31)


# Compact last level (gkm_msd.hip level_pass): k = 21 leaves 27 key bits below L1, so L1 stores
# (low bits, start) pairs + digit bytes and the finishing kernels rebuild the keys from the bucket
# prefixes; the periodic run makes sub-buckets above the local limit, which are expanded back for
# another global level.  GKM_NO_COMPACT=1 runs the same input with full keys everywhere.
@pytest.mark.parametrize("compact", [True, False])
def test_compact_level_with_big_sub_buckets_vs_oracle(compact, monkeypatch):
    if not compact:
        monkeypatch.setitem(_native.options, "GKM_NO_COMPACT", "1")
    rng = np.random.default_rng(21)
    seqs = random_genome(rng, [1_500_000, 400_000])
    seqs.append(("periodic", "ACGT" * 30_000 + "AACCGGTT" * 8_000))
    k = 21
    sc = SequenceCollection(sequence_list=seqs)
    km = gk.Kmers(sc, min_kmer_len=k, max_kmer_len=k)
    eng = km._get_engine()
    eng.profile_enable(True)
    km.sort()
    assert ("msd_pass_l1c" in str(eng.profile_report())) == compact
    eng.profile_enable(False)
    unsorted = oracle.enumerate_starts(sc.forward_sba, sc._forward_sba_seg_starts, k)
    want = oracle.quicksort(sc.forward_sba, unsorted, k, k, break_ties=True)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)
    # the keys the finishing kernels rebuilt (one-word keys: the sort's own, not a re-encode)
    spec = oracle.key_spec(True, k, k)
    np.testing.assert_array_equal(km.get_encoded_kmers(), oracle.encode_keys(sc.forward_sba, want, *spec))
    h, t = km.get_kmer_group_counts(k, max_counts_bin=64)
    oh, ot = oracle.group_scan(sc.forward_sba, want, k, max_counts_bin=64)
    np.testing.assert_array_equal(h, oh)
    assert t == ot


# Compact buckets of C3's wave class (257..512 k-mers): with a 6-bit L1 the compact level leaves
# buckets of ~490 k-mers for msd_wave_kernel<8> (C3's ~370 are in the same class), plus a periodic
# run whose sub-buckets outgrow the rank-by-count limit and are re-listed with rebuilt keys.
def test_compact_wave_class_vs_oracle(monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_LEVEL_BITS", "7,6,8")
    rng = np.random.default_rng(22)
    seqs = random_genome(rng, [3_000_000, 1_000_000])
    seqs.append(("periodic", "ACGTTGCA" * 5_000 + "AACCGGTTAC" * 3_000))
    k = 21
    sc = SequenceCollection(sequence_list=seqs)
    km = gk.Kmers(sc, min_kmer_len=k, max_kmer_len=k)
    eng = km._get_engine()
    eng.profile_enable(True)
    km.sort()
    rep = str(eng.profile_report())
    eng.profile_enable(False)
    assert "msd_pass_l1c" in rep and "msd_local_wave8" in rep
    unsorted = oracle.enumerate_starts(sc.forward_sba, sc._forward_sba_seg_starts, k)
    want = oracle.quicksort(sc.forward_sba, unsorted, k, k, break_ties=True)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)
    spec = oracle.key_spec(True, k, k)
    np.testing.assert_array_equal(km.get_encoded_kmers(), oracle.encode_keys(sc.forward_sba, want, *spec))
    h, t = km.get_kmer_group_counts(k, max_counts_bin=64)
    oh, ot = oracle.group_scan(sc.forward_sba, want, k, max_counts_bin=64)
    np.testing.assert_array_equal(h, oh)
    assert t == ot


def test_iupac_k31_vs_oracle():
    rng = np.random.default_rng(4)
    oracle_check(random_genome(rng, [120_000, 60_000], alphabet=b"ACGTACGTACGTNRY"), 31, 31)


@pytest.mark.parametrize("k", [1, 2, 5, 16, 32, 33, 63, 64, 100])
def test_k_sweep_vs_oracle(k):
    rng = np.random.default_rng(100 + k)
    oracle_check(random_genome(rng, [40_000, 9_000, 128]), k, k)


# Multi-word keys (2 bits x k > 64 or 4 bits x k > 64): the MSD sorts the first key word, then
# each group of equal earlier words by the next word (gkm_msd.hip next_phase).  Planted repeats
# make groups that tie on one and on every word.
@pytest.mark.parametrize("alphabet", [b"ACGT", b"ACGTACGTACGTNRY"])
@pytest.mark.parametrize("k", [17, 33, 40, 63, 64])
def test_multiword_repeats_vs_oracle(alphabet, k):
    rng = np.random.default_rng(200 + k + len(alphabet))
    rep = rng.choice(np.frombuffer(alphabet, dtype=np.uint8), 3000).astype(np.uint8)
    oracle_check(random_genome(rng, [60_000, 25_000, 300], alphabet=alphabet, repeat=rep, copies=6), k, k)


@pytest.mark.parametrize("alphabet", [b"ACGT", b"ACGTN"])
def test_multiword_big_first_word_group(alphabet):
    # 6000 contigs of one k-mer each that share their first 32 bases: a first-word group above the
    # local limit (4096) goes through a global level of the second phase; a few exact duplicates
    rng = np.random.default_rng(31)
    pre = "A" * 32
    tails = ["".join(rng.choice(list(alphabet.decode()), 31)) for _ in range(6000)]
    tails += tails[:50]
    oracle_check([(f"r{i}", pre + t) for i, t in enumerate(tails)], 63, 63)


def test_multiword_homopolymer_all_words_tie():
    seqs = [("a", "A" * 30_000), ("b", "C" * 64 + "A" * 9000), ("c", "ACGT" * 3000)]
    oracle_check(seqs, 63, 63)
    oracle_check(seqs, 40, 40)


@pytest.mark.parametrize("min_k,max_k", [(1, 8), (5, 31), (10, 40), (3, 70)])
def test_bounded_variable_length_vs_oracle(min_k, max_k):
    rng = np.random.default_rng(min_k * 7 + max_k)
    rep = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 300).astype(np.uint8)
    oracle_check(random_genome(rng, [30_000, 8_000, 500], repeat=rep, copies=5), min_k, max_k)


@pytest.mark.parametrize("alphabet", [b"ACGT", b"ACGTN"])
def test_suffix_mode_vs_oracle(alphabet):
    rng = np.random.default_rng(len(alphabet))
    rep = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 200).astype(np.uint8)
    oracle_check(random_genome(rng, [12_000, 3_000, 90], alphabet=alphabet, repeat=rep, copies=4), 2, None,
                 check_counts=False)


def test_long_bound_uses_doubling_vs_oracle():
    rng = np.random.default_rng(9)
    rep = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 400).astype(np.uint8)
    oracle_check(random_genome(rng, [20_000, 5_000], repeat=rep, copies=6), 10, 300)


def test_user_assigned_starts_sort_like_break_ties():
    rng = np.random.default_rng(11)
    seqs = random_genome(rng, [20_000])
    sc = SequenceCollection(sequence_list=seqs)
    km = gk.Kmers(sc, min_kmer_len=12, max_kmer_len=12)
    user = rng.permutation(km.kmer_sba_start_indices)[:5000].astype(np.uint32)
    user = np.concatenate([user, user[:100]])  # duplicates tie on key and index
    km.kmer_sba_start_indices = user
    km.sort()
    want = oracle.quicksort(sc.forward_sba, user, 12, 12, break_ties=True)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)
    # in-place semantics: the caller's array object now holds the sorted order
    np.testing.assert_array_equal(user, want)


def test_invalid_user_starts_raise_reference_assertion():
    sc = SequenceCollection(sequence_list=[("a", "ACGTACGT"), ("b", "GGGCCC")])
    km = gk.Kmers(sc, min_kmer_len=4, max_kmer_len=4)
    km.kmer_sba_start_indices = np.array([0, 6, 1], dtype=np.uint32)  # 6: only 2 bases before '$'
    with pytest.raises(AssertionError, match="kmers compared were less than min_kmer_len"):
        km.sort()


def test_custom_python_filter_is_honoured():
    rng = np.random.default_rng(12)
    sc = SequenceCollection(sequence_list=random_genome(rng, [5000]))
    km = gk.Kmers(sc, min_kmer_len=6, max_kmer_len=6)
    km.sort()

    def starts_with_a(sba, strand, idx):
        return sba[idx] == ord("A")

    got = km.get_kmer_count(6, starts_with_a)
    filt_starts = [s for s in km.kmer_sba_start_indices.tolist() if sc.forward_sba[s] == ord("A")]
    _, want = oracle.group_scan(sc.forward_sba, np.array(filt_starts, dtype=np.uint32), 6, max_counts_bin=10)
    assert got == want


FILTER_SPECS = [
    {"kind": "homopolymer", "max_homopolymer_size": 3, "kmer_len": 31},
    {"kind": "homopolymer", "max_homopolymer_size": 4, "kmer_len": 40},  # past some '$': raises
    {"kind": "gc", "min_gc": 0.35, "max_gc": 0.6, "kmer_len": 31},
    {"kind": "gc", "min_gc": 0.3, "max_gc": 0.7, "kmer_len": 36},  # raises (segment end)
    {"kind": "no_ambiguous", "kmer_len": 31},
    {"kind": "no_ambiguous", "kmer_len": 33},  # raises (segment end)
    {"kind": "length", "min_kmer_len": 31},
    {"kind": "crispr_ngg"},
]


@pytest.mark.parametrize("spec", FILTER_SPECS, ids=lambda s: "-".join(str(v) for v in s.values()))
def test_builtin_filters_per_position_vs_oracle(spec):
    """The built-in filters are evaluated once per sba position and gathered into sorted order
    (gkm_group.hip filter_pos_kernel): histograms, totals, yields and the raised error (its type
    and sba index: the first raising k-mer in sorted order) against the oracle's group scan over
    the same sorted starts, on an IUPAC sequence with N runs, several contigs and ragged ends."""
    rng = np.random.default_rng(21)
    rep = rng.choice(np.frombuffer(b"ACGTACGTGCCGGS", dtype=np.uint8), 900).astype(np.uint8)
    seqs = random_genome(rng, [60_000, 41_003, 25_017], alphabet=b"ACGTACGTACGTACGTNRY", repeat=rep, copies=6)
    seqs = [(n, s[:5000] + "N" * 700 + s[5000:]) for n, s in seqs]
    sc = SequenceCollection(sequence_list=seqs)
    km = gk.Kmers(sc, min_kmer_len=31, max_kmer_len=31)
    km.sort()
    sba, st = sc.forward_sba, km.kmer_sba_start_indices
    filt, params = filter_of(spec), oracle.filter_params(spec)
    try:
        want = oracle.group_scan(sba, st, 31, params, max_counts_bin=100)
    except oracle.OracleError as e:
        with pytest.raises((ValueError, IndexError)) as got:
            km.get_kmer_group_counts(31, filt, max_counts_bin=100)
        if "kmer_sba_start_idx" in str(got.value) or "sba index" in str(got.value):
            assert str(e.idx) in str(got.value)
        return
    h, t = km.get_kmer_group_counts(31, filt, max_counts_bin=100)
    assert h.tolist() == want[0].tolist() and int(t) == want[1]
    ys = oracle.group_scan(sba, st, 31, params, min_group_size=2, yield_first_n=2)
    got = list(km.get_kmers(31, kmer_filter_func=filt, min_group_size=2, yield_first_n=2))
    assert got == ys


def test_unique_counts_match_groups():
    rng = np.random.default_rng(13)
    rep = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 700).astype(np.uint8)
    km, sc, want = oracle_check(random_genome(rng, [50_000, 20_000], repeat=rep, copies=9), 25, 25)
    first, counts = km.get_unique_kmers()
    ys = oracle.group_scan(sc.forward_sba, want, 25, yield_first_n=1)
    assert first.tolist() == [y[0] for y in ys]
    assert counts.tolist() == [y[2] for y in ys]
    assert int(counts.sum()) == len(want)


@pytest.mark.parametrize("shape", ["one_group", "all_distinct", "mixed_runs", "sparse_heads"])
def test_unique_counts_many_tiles(shape):
    """gk_unique_counts' one-pass selection (look-back over 4096-flag tiles, 16-byte output groups)
    at sizes with thousands of tiles: runs of head-less tiles longer than one look-back window,
    every position a head, and ragged mixtures; first index + multiplicity vs numpy on the keys."""
    rng = np.random.default_rng(hash(shape) % 1000)
    k = 31
    if shape == "one_group":
        s = np.full(3_000_000, ord("A"), np.uint8)
    elif shape == "all_distinct":
        s = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, 2_500_000)].copy()
    elif shape == "mixed_runs":
        s = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, 3_000_000)].copy()
        for L in (40, 300, 5000, 70_000, 400_000):  # homopolymer runs: groups of L - k + 1
            p = int(rng.integers(0, len(s) - L))
            s[p:p + L] = ord("C")
        rep = s[:2000].copy()
        for p in rng.integers(0, len(s) - 2000, 50):
            s[p:p + 2000] = rep
    else:  # few distinct k-mers: long head-less stretches between heads
        s = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, 3_000_000)].copy()
        s[:] = np.repeat(s[::50_000], 50_000)[:len(s)]
    e = _native.Engine()
    e.set_sequence(s, np.array([0], np.uint32))
    e.enumerate(k)
    e.sort(k)
    keys = e.copy_keys()
    n = e.n
    flat = keys.reshape(n, -1)
    head = np.ones(n, dtype=bool)
    head[1:] = (flat[1:] != flat[:-1]).any(axis=1)
    want_first = np.flatnonzero(head)
    want_cnt = np.diff(np.append(want_first, n))
    first, counts = e.unique_counts()
    np.testing.assert_array_equal(first, want_first)
    np.testing.assert_array_equal(counts, want_cnt)


@pytest.mark.parametrize("k,canonical", [(31, False), (31, True), (63, False)])
def test_big_groups_of_identical_kmers(k, canonical):
    """Groups of identical k-mers larger than a local bucket (poly-A, (CA)n and a 300-bp unit in
    thousands of exact copies) inside a genome large enough that the MSD driver sends them from the
    next-level list straight to the done list (drop_uniform) instead of partitioning them level by
    level: starts, keys and unique counts vs the oracle."""
    rng = np.random.default_rng(77 + k)
    s = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, 3_200_000)].copy()
    s[100_000:110_000] = ord("A")
    s[500_000:514_000] = np.frombuffer(b"CA" * 7000, dtype=np.uint8)
    unit = s[900_000:900_300].copy()
    for p in range(1_000_000, 1_000_000 + 6000 * 300, 300):
        s[p:p + 300] = unit
    seg = np.array([0], dtype=np.uint32)
    e = _native.Engine()
    e.set_sequence(s, seg)
    e.enumerate(k)
    e.sort(k, canonical=canonical)
    unsorted = oracle.enumerate_starts(s, seg, k)
    if canonical:
        want = oracle.canonical_sort(s, unsorted, k)
        keys = oracle.canonical_keys(s, want, k, 2)
    else:
        want = oracle.quicksort(s, unsorted, k, k, break_ties=True)
        keys = oracle.encode_keys(s, want, *oracle.key_spec(True, k, k))
    np.testing.assert_array_equal(e.copy_starts(), want)
    got = e.copy_keys()
    np.testing.assert_array_equal(got, keys.reshape(got.shape))
    flat = got.reshape(len(got), -1)
    head = np.ones(len(flat), dtype=bool)
    head[1:] = (flat[1:] != flat[:-1]).any(axis=1)
    first, counts = e.unique_counts()
    np.testing.assert_array_equal(first, np.flatnonzero(head))
    np.testing.assert_array_equal(counts, np.diff(np.append(np.flatnonzero(head), len(flat))))
    assert counts.max() >= 5000  # the groups the test is about


def test_single_kmer_and_tiny_inputs():
    sc = SequenceCollection(sequence_list=[("a", "ACGTA")])
    km = gk.Kmers(sc, min_kmer_len=5, max_kmer_len=5)
    km.sort()
    assert km.kmer_sba_start_indices.tolist() == [0]
    assert km.get_kmer_group_counts(5, max_counts_bin=3)[0].tolist() == [0, 1, 0, 0]
    sc = SequenceCollection(sequence_list=[("a", "A")])
    km = gk.Kmers(sc)
    km.sort()
    assert km.kmer_sba_start_indices.tolist() == [0]


# ---------------------------------------------------------------------------------------------
# size-independent properties at a large size
# ---------------------------------------------------------------------------------------------
def test_large_single_contig_properties():
    L = 100_000_000
    rng = np.random.default_rng(42)
    sba = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, L)]
    sc = SequenceCollection()
    sc.forward_sba = sba
    sc._forward_sba_seg_starts = np.zeros(1, dtype=np.uint32)
    sc.forward_record_names = ["chr0"]
    sc._strands_loaded = "forward"
    km = gk.Kmers(sc, min_kmer_len=31, max_kmer_len=31)
    km.sort()
    starts = km.kmer_sba_start_indices
    n = L - 30
    assert starts.shape == (n,)
    # permutation of the enumerate output
    assert np.array_equal(np.bincount(starts, minlength=n), np.ones(n, dtype=np.int64))
    keys = km.get_encoded_kmers()[:, 0]
    assert np.all(keys[1:] >= keys[:-1])
    ties = keys[1:] == keys[:-1]
    assert np.all(starts[1:][ties] > starts[:-1][ties])
    # spot-check keys against the encoding of the sba
    idx = rng.integers(0, n, 10_000)
    np.testing.assert_array_equal(oracle.encode_keys(sba, starts[idx], 2, 31, 0, 1)[:, 0], keys[idx])
    first, counts = km.get_unique_kmers()
    assert int(counts.sum()) == n
    h, t = km.get_kmer_group_counts(31, max_counts_bin=8)
    assert t == n and int((h * np.arange(9))[:8].sum()) <= n


# ---------------------------------------------------------------------------------------------
# get_kmers(kmer_info_to_yield="full"): device gk_locate vs the per-k-mer reference path
# ---------------------------------------------------------------------------------------------
def _full_info_reference(km, kmer_len, one_based, **kw):
    """kmers.py:1180-1264 element by element: the minimum info, then get_kmer_info per k-mer."""
    info = km.generate_get_kmer_info_func(one_based)
    starts = km.kmer_sba_start_indices
    out = []
    try:
        for num, y, t in km.get_kmers(kmer_len, kmer_info_to_yield="minimum", **kw):
            out.append(info(num, starts, km.seq_coll.forward_sba, kmer_len, y, t))
    except ValueError as e:
        out.append(("ValueError", str(e)))
    return out


def _full_info_device(km, kmer_len, one_based, **kw):
    out = []
    try:
        for t in km.get_kmers(kmer_len, one_based_seq_index=one_based, kmer_info_to_yield="full", **kw):
            out.append(t)
    except ValueError as e:
        out.append(("ValueError", str(e)))
    return out


@pytest.mark.parametrize("sort", [True, False])
@pytest.mark.parametrize("kmer_len,one_based,kw", [
    (8, False, {}), (8, True, {"min_group_size": 2}), (5, False, {"yield_first_n": 2}),
    (None, False, {}), (12, True, {"max_group_size": 3}),
])
def test_full_info_matches_reference_path(sort, kmer_len, one_based, kw):
    rng = np.random.default_rng(21)
    seqs = random_genome(rng, [3000, 40, 1200, 9], alphabet=b"ACGT")
    seqs = [(n, s[: len(s) // 3] + s[: len(s) // 3] + s[len(s) // 3:]) for n, s in seqs]  # planted repeats
    sc = SequenceCollection(sequence_list=seqs)
    km = gk.Kmers(sc, min_kmer_len=8, max_kmer_len=None if kmer_len is None else 12)
    if sort:
        km.sort()
    if not sort and kw:
        pytest.skip("group-size arguments need a sorted Kmers")
    want = _full_info_reference(km, kmer_len, one_based, **kw)
    got = _full_info_device(km, kmer_len, one_based, **kw)
    assert got == want


@pytest.mark.parametrize("k,alphabet", [(63, b"ACGT"), (31, b"ACGTN")])
def test_multiword_runs_the_msd_phases(k, alphabet):
    """Fixed-length multi-word keys are sorted by the MSD path (no LSD fallback): the profile
    shows the L0 pass and the tie re-encode of the second phase."""
    rng = np.random.default_rng(5)
    rep = rng.choice(np.frombuffer(alphabet, dtype=np.uint8), 2000).astype(np.uint8)
    sc = SequenceCollection(sequence_list=random_genome(rng, [50_000], alphabet=alphabet, repeat=rep, copies=3))
    km = gk.Kmers(sc, min_kmer_len=k, max_kmer_len=k)
    eng = km._get_engine()
    eng.profile_enable(True)
    km.sort()
    rep_ = eng.profile_report()
    assert "msd_pass_l0" in str(rep_) and "msd_tie_encode" in str(rep_), rep_
    want = oracle.quicksort(sc.forward_sba, oracle.enumerate_starts(sc.forward_sba, sc._forward_sba_seg_starts, k),
                            k, k, break_ties=True)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)


def test_multiword_many_tiny_tie_groups_flat_encode():
    """4-bit keys at k=31 over a low-entropy alphabet: the first word (16 symbols) ties often, so
    the second phase sees >4096 small groups (flat re-encode, one-thread tiny buckets)."""
    rng = np.random.default_rng(77)
    seqs = random_genome(rng, [1_500_000, 500_000], alphabet=b"ACACACACACN")
    seqs.append(("n", "N" * 3000 + "ACGT" * 100))  # one large all-N group
    oracle_check(seqs, 31, 31)


def n_run_genome(rng, lengths, runs=6, run_len=(40, 400), sparse=30):
    """Random ACGT records with N runs (GRCh38-like) and a few scattered IUPAC letters, planted
    repeats inside and across records."""
    rep = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 900).astype(np.uint8)
    seqs = []
    for i, L in enumerate(lengths):
        s = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), L).astype(np.uint8)
        for _ in range(3):
            at = int(rng.integers(0, max(1, L - len(rep))))
            s[at:at + len(rep)] = rep[: L - at]
        for _ in range(runs):
            a = int(rng.integers(0, L))
            s[a:a + int(rng.integers(*run_len))] = ord("N")
        at = rng.integers(0, L, sparse)
        s[at] = np.frombuffer(b"RYKMSWBDHVN", dtype=np.uint8)[rng.integers(0, 11, sparse)]
        s[:50] = ord("N")  # contig starts / ends in N, as GRCh38's do
        s[-50:] = ord("N")
        seqs.append((f"c{i}", s.tobytes().decode()))
    return seqs


@pytest.mark.parametrize("k", [5, 21, 31, 32, 33, 63, 64])
def test_split_acgt_and_n_kmers_vs_oracle(k):
    """Mixed sba with few non-ACGT k-mers: ACGT-only k-mers on the 2-bit MSD, the rest on 4-bit keys,
    merged (gkm_split.hip) -- the profile shows the merge ran."""
    rng = np.random.default_rng(500 + k)
    seqs = n_run_genome(rng, [120_000, 40_000, 3_000])
    sc = SequenceCollection(sequence_list=seqs)
    km = gk.Kmers(sc, min_kmer_len=k, max_kmer_len=k)
    eng = km._get_engine()
    eng.profile_enable(True)
    km.sort()
    assert "split_merge" in str(eng.profile_report())
    unsorted = oracle.enumerate_starts(sc.forward_sba, sc._forward_sba_seg_starts, k)
    want = oracle.quicksort(sc.forward_sba, unsorted, k, k, break_ties=True)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)
    h, t = km.get_kmer_group_counts(k, max_counts_bin=64)
    oh, ot = oracle.group_scan(sc.forward_sba, want, k, max_counts_bin=64)
    np.testing.assert_array_equal(h, oh)
    assert t == ot
    spec = oracle.key_spec(False, k, k)
    np.testing.assert_array_equal(km.get_encoded_kmers(), oracle.encode_keys(sc.forward_sba, want, *spec))


@pytest.mark.gpu
@pytest.mark.parametrize("k", [5, 31, 63])
def test_split_homopolymer_runs_of_several_letters_vs_oracle(k):
    """Runs of several non-ACGT letters (N, R, Y, K, W) longer than k: their homopolymer k-mers
    skip the B sort as one group per letter and are spliced into the sorted B run at their
    insertion points (gkm_split.hip); scattered letters keep some non-homopolymer B k-mers."""
    rng = np.random.default_rng(900 + k)
    seqs = n_run_genome(rng, [60_000, 25_000], runs=2)
    out = []
    for name, s in seqs:
        b = bytearray(s.encode())
        for letter in b"NRYKW":
            for a in rng.integers(100, len(b) - 500, 2):
                n_run = int(rng.integers(k + 1, k + 300))
                b[a:a + n_run] = bytes([letter]) * n_run
        out.append((name, b.decode()))
    sc = SequenceCollection(sequence_list=out)
    km = gk.Kmers(sc, min_kmer_len=k, max_kmer_len=k)
    eng = km._get_engine()
    eng.profile_enable(True)
    km.sort()
    assert "split_b_homo" in str(eng.profile_report())
    unsorted = oracle.enumerate_starts(sc.forward_sba, sc._forward_sba_seg_starts, k)
    want = oracle.quicksort(sc.forward_sba, unsorted, k, k, break_ties=True)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)
    h, t = km.get_kmer_group_counts(k, max_counts_bin=64)
    oh, ot = oracle.group_scan(sc.forward_sba, want, k, max_counts_bin=64)
    np.testing.assert_array_equal(h, oh)
    assert t == ot
    spec = oracle.key_spec(False, k, k)
    np.testing.assert_array_equal(km.get_encoded_kmers(), oracle.encode_keys(sc.forward_sba, want, *spec))


def _split_keys_check(seqs, k, canonical=False):
    """Through the engine (gk_enumerate / gk_sort / gk_copy_keys): records shorter than k are legal
    there, while Kmers.__init__ rejects them (kmers.py:744-749)."""
    sc = SequenceCollection(sequence_list=seqs)
    sba, seg = sc.forward_sba, sc._forward_sba_seg_starts
    e = _native.Engine()
    e.set_sequence(sba, seg)
    e.enumerate(k)
    e.sort(k, canonical=canonical)
    unsorted = oracle.enumerate_starts(sba, seg, k)
    if canonical:
        want = oracle.canonical_sort(sba, unsorted, k)
        keys = oracle.canonical_keys(sba, want, k, 4)
    else:
        want = oracle.quicksort(sba, unsorted, k, k, break_ties=True)
        keys = oracle.encode_keys(sba, want, *oracle.key_spec(False, k, k))
    np.testing.assert_array_equal(e.copy_starts(), want)
    np.testing.assert_array_equal(e.copy_keys(), keys)
    first, counts = e.unique_counts()
    assert int(counts.sum()) == len(want)


@pytest.mark.parametrize("k", [5, 20, 31])
def test_split_only_class_b_kmers_keys(k):
    """Every k-mer holds a non-ACGT letter (the split sort has no class-A k-mer): the keys come from
    the B sort and the homopolymer groups' constant keys."""
    rng = np.random.default_rng(80 + k)
    s = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, 20_000)].copy()
    s[::max(2, k // 2)] = ord("N")  # a non-ACGT byte in every window
    s[5000:5000 + 3 * k] = ord("R")
    _split_keys_check([("a", s.tobytes().decode())], k)


@pytest.mark.parametrize("k,canonical", [(31, False), (21, True), (32, True)])
def test_split_keys_with_homopolymers(k, canonical):
    rng = np.random.default_rng(95 + k)
    seqs = n_run_genome(rng, [40_000, 9_000], runs=3)
    out = []
    for name, s in seqs:
        b = bytearray(s.encode())
        for letter in b"NYR":
            a = int(rng.integers(100, len(b) - 400))
            b[a:a + k + 40] = bytes([letter]) * (k + 40)
        out.append((name, b.decode()))
    _split_keys_check(out, k, canonical)


# the 11-bit L0 (msd0_wide_kernel, GKM_WIDE_L0=1) with its 1024-thread block-local finishing class:
# random, repeat-heavy and multi-contig inputs, bit-exact against the oracle
@pytest.mark.parametrize("case", ["random", "block32", "repeats", "contigs", "homopolymer"])
def test_wide_l0_vs_oracle(case, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_WIDE_L0", "1")
    rng = np.random.default_rng(21)
    if case == "random":
        seqs = random_genome(rng, [1_500_000])
    elif case == "block32":  # ~5.9 K k-mers per 11-bit L0 bucket: the 1024-thread block class
        seqs = random_genome(rng, [12_000_000])
    elif case == "repeats":
        rep = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 9000).astype(np.uint8)
        seqs = random_genome(rng, [600_000, 300_000], repeat=rep, copies=9)
    elif case == "contigs":
        seqs = random_genome(rng, [40_000, 31, 250_000, 32, 99_999, 64])
    else:
        seqs = [("a", "A" * 40_000 + "C" * 9_000), ("b", "AC" * 30_000)]
    oracle_check(seqs, 31, 31)


@pytest.mark.parametrize("k", [12, 20, 32])
def test_wide_l0_k_sweep_vs_oracle(k, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_WIDE_L0", "1")
    rng = np.random.default_rng(k)
    oracle_check(random_genome(rng, [700_000, 12_345]), k, k)


# Packed-pair levels (gkm_msd.hip level_pass, MODE 5): the level before a compact one writes
# (key bits below the sorted ones, start) in 10 bytes; the compact level reads them (IN79), the
# buckets the pair level sends to the finishing classes and a next level that is not compact get
# (key, start) back first (expand_pair_*).  At test sizes GKM_TEST_PAIRS=1 makes every level whose
# remaining bits fit write pairs; the low-entropy input keeps buckets big for several levels.
@pytest.mark.parametrize("level_bits,k", [("8", 31), ("8,6", 31), ("7,8,8", 31), ("7,8,8", 24), ("8", 32),
                                          ("6,8,8", 31), ("6,8,8", 27)])
def test_packed_pair_levels_vs_oracle(level_bits, k, monkeypatch):
    # k = 24 / 32: 33 / 48 key bits left behind the pair level (the two ends of its range)
    monkeypatch.setitem(_native.options, "GKM_TEST_PAIRS", "1")
    monkeypatch.setitem(_native.options, "GKM_LEVEL_BITS", level_bits)
    rng = np.random.default_rng(31)
    seqs = random_genome(rng, [1_600_000, 800_000], alphabet=b"AC")
    seqs.append(("mixed", random_genome(rng, [300_000])[0][1]))
    km, sc, want = oracle_check(seqs, k, k)
    spec = oracle.key_spec(True, k, k)
    np.testing.assert_array_equal(km.get_encoded_kmers(), oracle.encode_keys(sc.forward_sba, want, *spec))


# The packed L0 (P88, round 5): the L0 writes each element as its level-1 digit byte, a packed pair
# (key bits below that digit above the start's high bits) and the start's low bits -- 11 B instead
# of 13 -- and the level behind it reads that form (INP = 2) when it writes packed pairs itself;
# otherwise the big buckets are expanded back to (key, start) first (expand_p88_kernel), and L0
# buckets small enough to finish locally always are (expand_p88_list_kernel).  At test sizes
# GKM_TEST_P88=1 makes the L0 pack wherever the bits fit; GKM_TEST_PAIRS=1 makes the next level
# write pairs (so it reads the packed form); low-entropy input keeps buckets big for several levels,
# random input sends most L0 buckets to the local classes.
@pytest.mark.parametrize("pairs", [True, False], ids=["l1_pairs", "l1_plain"])
@pytest.mark.parametrize("alphabet,k,level_bits", [(b"AC", 31, None), (b"AC", 24, None), (b"ACGT", 31, None),
                                                   (b"AC", 31, "8,8,8"), (b"AC", 32, "8,8,8"), (b"AC", 31, "6,8,8"),
                                                   (b"ACGT", 31, "6,8,8")])
def test_packed_l0_vs_oracle(pairs, alphabet, k, level_bits, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_TEST_P88", "1")
    if pairs:
        monkeypatch.setitem(_native.options, "GKM_TEST_PAIRS", "1")
    if level_bits:
        monkeypatch.setitem(_native.options, "GKM_LEVEL_BITS", level_bits)
    rng = np.random.default_rng(k + len(alphabet))
    seqs = random_genome(rng, [1_600_000, 700_000], alphabet=alphabet)
    seqs.append(("mixed", random_genome(rng, [250_000])[0][1]))
    km, sc, want = oracle_check(seqs, k, k)
    spec = oracle.key_spec(True, k, k)
    np.testing.assert_array_equal(km.get_encoded_kmers(), oracle.encode_keys(sc.forward_sba, want, *spec))


@pytest.mark.parametrize("pairs", [True, False], ids=["l1_pairs", "l1_plain"])
def test_packed_l0_canonical_vs_oracle(pairs, monkeypatch):
    # canonical 64-bit first words (k = 32): the 8-bit L0 leaves 56 bits, 48 of them in the pair
    monkeypatch.setitem(_native.options, "GKM_TEST_P88", "1")
    if pairs:
        monkeypatch.setitem(_native.options, "GKM_TEST_PAIRS", "1")
    rng = np.random.default_rng(5)
    s = np.frombuffer(b"ACG", dtype=np.uint8)[rng.integers(0, 3, 1_500_000)].copy()
    seg = np.array([0], dtype=np.uint32)
    e = _native.Engine()
    e.set_sequence(s, seg)
    n = e.enumerate(32)
    e.sort(32, canonical=True)
    want = oracle.canonical_sort(s, oracle.enumerate_starts(s, seg, 32), 32)
    np.testing.assert_array_equal(e.copy_starts(np.empty(n, dtype=np.uint32)), want)
    got = e.copy_keys()
    keys = oracle.canonical_keys(s, want, 32, 2)
    np.testing.assert_array_equal(got, keys.reshape(got.shape))


# The packed L0 under multi-word keys (round 5): phase 0 sorts the first word through it, the tie
# phases then read keys[0] / vals[0] as usual.  Planted repeats tie first words (k = 45, 63), and an
# N run makes the 4-bit split path sort its ACGT-only class on 2-bit keys through the packed L0.
@pytest.mark.parametrize("pairs", [True, False], ids=["l1_pairs", "l1_plain"])
@pytest.mark.parametrize("k", [45, 63])
@pytest.mark.parametrize("canonical", [False, True], ids=["fwd", "canon"])
def test_packed_l0_multiword_vs_oracle(pairs, k, canonical, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_TEST_P88", "1")
    if pairs:
        monkeypatch.setitem(_native.options, "GKM_TEST_PAIRS", "1")
    rng = np.random.default_rng(k + 2 * canonical)
    s = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, 1_200_000)].copy()
    rep = s[1000:1000 + 4000].copy()
    for at in (100_000, 400_000, 800_000):
        s[at:at + 4000] = rep
    seg = np.array([0], dtype=np.uint32)
    e = _native.Engine()
    e.set_sequence(s, seg)
    n = e.enumerate(k)
    e.sort(k, canonical=canonical)
    starts = oracle.enumerate_starts(s, seg, k)
    want = oracle.canonical_sort(s, starts, k) if canonical else oracle.quicksort(s, starts, k, k, break_ties=True)
    np.testing.assert_array_equal(e.copy_starts(np.empty(n, dtype=np.uint32)), want)
    got = e.copy_keys()
    keys = oracle.canonical_keys(s, want, k, 2) if canonical else oracle.encode_keys(s, want, *oracle.key_spec(True, k, k))
    np.testing.assert_array_equal(got, keys.reshape(got.shape))


@pytest.mark.parametrize("canonical", [False, True], ids=["fwd", "canon"])
def test_packed_l0_split_vs_oracle(canonical, monkeypatch):
    # an N run: 4-bit keys, the ACGT-only class sorted on 2-bit keys (63 symbols: two words)
    monkeypatch.setitem(_native.options, "GKM_TEST_P88", "1")
    monkeypatch.setitem(_native.options, "GKM_TEST_PAIRS", "1")
    rng = np.random.default_rng(11 + canonical)
    s = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, 900_000)].copy()
    s[300_000:300_500] = ord("N")
    s[600_000:600_003] = ord("R")
    seg = np.array([0], dtype=np.uint32)
    e = _native.Engine()
    e.set_sequence(s, seg)
    n = e.enumerate(63)
    e.sort(63, canonical=canonical)
    starts = oracle.enumerate_starts(s, seg, 63)
    want = oracle.canonical_sort(s, starts, 63) if canonical else oracle.quicksort(s, starts, 63, 63, break_ties=True)
    np.testing.assert_array_equal(e.copy_starts(np.empty(n, dtype=np.uint32)), want)


# Round 5: on a mixed sba the split sort's merge writes the 4-bit keys of the ACGT-only k-mers of
# k = 33..63 from a 2-bit packed copy of the sequence (gkm_split.hip put_key4_packed) instead of a
# re-encode after the sort; W = 3 (k <= 48) and 4 words, forward and canonical, N runs (homopolymer
# groups) and scattered IUPAC letters (the class-B rest), several contigs
@pytest.mark.parametrize("k", [33, 40, 48, 49, 63])
@pytest.mark.parametrize("canonical", [False, True], ids=["fwd", "canon"])
@pytest.mark.parametrize("transfer", ["plain", "packed"])
def test_split_merge_packed_keys_vs_oracle(k, canonical, transfer, monkeypatch):
    # transfer "packed": the sequence goes through the packed transfer (GKM_PACK_MIN=0), whose
    # resident packed copy the merge then reads instead of packing the sequence itself
    if transfer == "packed":
        monkeypatch.setenv("GKM_PACK_MIN", "0")
        monkeypatch.setenv("GKM_PACK_BLOCKS", "1")
    rng = np.random.default_rng(100 + k + canonical)
    s = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, 700_000)].copy()
    s[100_000:100_400] = ord("N")
    s[300_000:300_090] = ord("N")
    s[450_000:450_200:13] = ord("R")
    s[520_000:520_004] = ord("Y")
    s[600_000:604_000] = s[10_000:14_000]  # repeats: ties in the first word
    s[250_000] = ord("$")
    s[500_000] = ord("$")
    seg = np.array([0, 250_001, 500_001], dtype=np.uint32)
    e = _native.Engine()
    e.set_sequence(s, seg)
    n = e.enumerate(k)
    e.sort(k, canonical=canonical)
    starts = oracle.enumerate_starts(s, seg, k)
    want = oracle.canonical_sort(s, starts, k) if canonical else oracle.quicksort(s, starts, k, k, break_ties=True)
    np.testing.assert_array_equal(e.copy_starts(np.empty(n, dtype=np.uint32)), want)
    got = e.copy_keys()
    keys = oracle.canonical_keys(s, want, k, 4) if canonical else oracle.encode_keys(s, want, *oracle.key_spec(False, k, k))
    np.testing.assert_array_equal(got, keys.reshape(got.shape))
    # the same keys through the re-encode after the sort
    monkeypatch.setitem(_native.options, "GKM_NO_MERGE_KEYS", "1")
    e2 = _native.Engine()
    e2.set_sequence(s, seg)
    e2.enumerate(k)
    e2.sort(k, canonical=canonical)
    np.testing.assert_array_equal(e2.copy_keys(), got)


# Whole-array sorts of encoded keys (bounded variable length, IUPAC 4-bit keys, the prefix-doubling
# seeds and rank pairs) take the MSD levels over the keys from 2^20 keys on (msd_sort_keys);
# GKM_MSD_KEYS_MIN lowers that bound so these sizes run it, GKM_SORT_KEYS_LSD=1 the LSD passes.
# Bounds of 30..64 on ACGT data take the capped doubling, whose first round shifts by
# min(29, max - 29) and reads seed keys of p + shift (the 3000-base repeats keep groups tied)
@pytest.mark.parametrize("path", ["msd", "lsd"])
@pytest.mark.parametrize("alphabet,min_k,max_k", [(b"ACGT", 5, 20), (b"ACGT", 1, None), (b"ACGTNRYKM", 3, 12),
                                                  (b"ACGTN", 2, None), (b"AC", 4, 29), (b"ACGT", 1, 50),
                                                  (b"ACGT", 1, 10), (b"ACGT", 1, 30), (b"AC", 2, 41),
                                                  (b"ACGT", 3, 64)])
def test_sort_keys_paths_vs_oracle(path, alphabet, min_k, max_k, monkeypatch):
    if path == "msd":
        monkeypatch.setitem(_native.options, "GKM_MSD_KEYS_MIN", "2048")
    else:
        monkeypatch.setitem(_native.options, "GKM_SORT_KEYS_LSD", "1")
    rng = np.random.default_rng(min_k * 7 + (max_k or 0))
    rep = rng.choice(np.frombuffer(alphabet, dtype=np.uint8), 3000).astype(np.uint8)
    oracle_check(random_genome(rng, [60_000, 20_000, 7_000, 40], alphabet=alphabet, repeat=rep, copies=3),
                 min_k, max_k)


# user-provided starts under max_kmer_len=None: the doubling ranks every position, then sorts the
# given starts by their final rank (the non-enumerated branch), on the tied-group MSD path
@pytest.mark.parametrize("path", ["msd", "lsd"])
def test_doubling_user_starts_vs_oracle(path, monkeypatch):
    if path == "msd":
        monkeypatch.setitem(_native.options, "GKM_MSD_KEYS_MIN", "2048")
    else:
        monkeypatch.setitem(_native.options, "GKM_SORT_KEYS_LSD", "1")
    rng = np.random.default_rng(77)
    rep = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 2000).astype(np.uint8)
    seqs = random_genome(rng, [30_000, 9_000, 300], repeat=rep, copies=4)
    sc = SequenceCollection(sequence_list=seqs)
    km = gk.Kmers(sc, min_kmer_len=3, max_kmer_len=None)
    user = rng.permutation(km.kmer_sba_start_indices)[:15_000].astype(km.kmer_sba_start_indices.dtype)
    km.kmer_sba_start_indices = user.copy()
    km.sort()
    want = oracle.quicksort(sc.forward_sba, np.sort(user, kind="stable"), 3, None, break_ties=True)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)


# a subset of user-given starts under a bounded 2-word key (min < max, max 30..64) keeps the direct
# keys: the capped doubling ranks every position of the sequence, which pays only when the starts
# cover most of them (round-4 advice); the encode stage then sees the user's starts, not every position
@pytest.mark.parametrize("max_k", [30, 41, 64])
def test_bounded_user_subset_keeps_direct_keys(max_k, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_MSD_KEYS_MIN", "2")
    rng = np.random.default_rng(max_k)
    sc = SequenceCollection(sequence_list=random_genome(rng, [40_000, 9_000, 300]))
    km = gk.Kmers(sc, min_kmer_len=20, max_kmer_len=max_k)
    user = rng.permutation(km.kmer_sba_start_indices)[:5_000].astype(km.kmer_sba_start_indices.dtype)
    km.kmer_sba_start_indices = user.copy()
    km._engine.profile_enable(True)
    km.sort()
    rep = km._engine.profile_report()
    km._engine.profile_enable(False)
    assert rep["encode"]["units"] == len(user), rep.get("encode")
    want = oracle.quicksort(sc.forward_sba, np.sort(user, kind="stable"), 20, max_k, break_ties=True)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)
    spec = oracle.key_spec(True, 20, max_k)
    assert km._engine.key_layout() == (spec[3], spec[0], spec[1])
    np.testing.assert_array_equal(km.get_encoded_kmers(), oracle.encode_keys(sc.forward_sba, want, *spec))


# the whole enumeration under a bounded 2-word key is sorted by capped doubling on the large-array
# route (keys are ranks inside the sort); the key contract stays the direct encoding, re-derived
# from the sorted starts when asked for, as on small arrays (round-4 advice)
@pytest.mark.parametrize("case", [c for c in CASES if c["max_kmer_len"] is not None], ids=lambda c: c["name"])
def test_encoded_keys_on_large_array_routes(case, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_MSD_KEYS_MIN", "2")
    km, a = make(case)
    km.sort()
    words, bits, symbols = km._engine.key_layout()
    if bits == 0:
        pytest.skip("bound beyond 256-bit keys: sorted by prefix doubling, keys are ranks")
    spec = oracle.key_spec(km._engine.is_acgt(), case["min_kmer_len"], case["max_kmer_len"])
    assert (words, bits, symbols) == (spec[3], spec[0], spec[1])
    np.testing.assert_array_equal(km.get_encoded_kmers(), oracle.encode_keys(a["sba"], a["starts_stable"], *spec))


# the golden cases again with the large-array routes forced at their sizes (GKM_MSD_KEYS_MIN=2):
# MSD levels over the keys, doubling by tied groups, and bounded keys of two or more words through
# capped doubling (keys become ranks) -- sorted starts and every query against the reference's
# answers
@pytest.mark.parametrize("case", CASES, ids=CASE_IDS)
def test_golden_on_large_array_routes(case, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_MSD_KEYS_MIN", "2")
    km, a = make(case)
    km.sort()
    np.testing.assert_array_equal(km.kmer_sba_start_indices, a["starts_stable"])
    for q, want in zip(case["queries"], case["results_stable_order"]):
        assert run_query(km, q) == want, q
