"""Device canonical k-mers (C5: Kmers.sort(canonical=True), GK_SORT_CANONICAL) vs the oracle.

The reference defines no canonical k-mer (kmers.py:689-696), so the order is this build's
extension and its parity is pinned to oracle.canonical_* (a numpy restatement built on the
reference's complement mapping, which tests/test_oracle_golden.py pins to golden vectors of the
reference's own reverse_complement_sba).  Bit-exact: starts, keys, strands, group histograms.
"""

import numpy as np
import pytest

from genome_kmers import _native
from genome_kmers import kmers as gk
from genome_kmers.sequence_collection import SequenceCollection
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert _native.device_count() > 0, "gpu tests need a visible MI355X"


def genome_with_rc_repeats(rng, lengths, alphabet, k_rep=2500, copies=4):
    """Random records with a planted repeat in both orientations (canonical ties across strands)
    and a few reverse-complement palindromes."""
    a = np.frombuffer(alphabet, dtype=np.uint8)
    rep = rng.choice(a, k_rep).astype(np.uint8)
    rc = oracle.reverse_complement(rep)
    pal_half = rng.choice(a, 40).astype(np.uint8)
    pal = np.concatenate([pal_half, oracle.reverse_complement(pal_half)])
    seqs = []
    for i, L in enumerate(lengths):
        s = rng.choice(a, L).astype(np.uint8)
        for c in range(copies):
            src = rep if c % 2 == 0 else rc
            at = int(rng.integers(0, max(1, L - len(src))))
            s[at:at + len(src)] = src[: L - at]
        at = int(rng.integers(0, max(1, L - len(pal))))
        s[at:at + len(pal)] = pal[: L - at]
        seqs.append((f"c{i}", s.tobytes().decode()))
    return seqs


def check_canonical(seqs, k, user_starts=None):
    sc = SequenceCollection(sequence_list=seqs)
    km = gk.Kmers(sc, min_kmer_len=k, max_kmer_len=k)
    starts = km.kmer_sba_start_indices.copy() if user_starts is None else user_starts
    if user_starts is not None:
        km.kmer_sba_start_indices = user_starts.copy()
    km.sort(canonical=True)
    got = km.kmer_sba_start_indices
    want = oracle.canonical_sort(sc.forward_sba, np.sort(starts, kind="stable"), k)
    np.testing.assert_array_equal(got, want)
    bits = 2 if km._engine.is_acgt() else 4
    np.testing.assert_array_equal(km.get_encoded_kmers(), oracle.canonical_keys(sc.forward_sba, want, k, bits))
    _, is_rc = oracle.canonical_windows(sc.forward_sba, want, k)
    np.testing.assert_array_equal(km.get_canonical_strands(), is_rc.astype(np.uint8))
    h, t = km.get_kmer_group_counts(k, max_counts_bin=32)
    oh, ot = oracle.canonical_group_hist(sc.forward_sba, want, k, 32)
    np.testing.assert_array_equal(h, oh)
    assert t == ot
    first, counts = km.get_unique_kmers()
    assert int(counts.sum()) == len(want) and len(first) == int(oh.sum())
    return km, sc


@pytest.mark.parametrize("k", [1, 5, 21, 31, 32, 33, 63, 64, 100])
def test_canonical_acgt_vs_oracle(k):
    rng = np.random.default_rng(300 + k)
    check_canonical(genome_with_rc_repeats(rng, [40_000, 12_000, 200], b"ACGT"), k)


@pytest.mark.parametrize("k", [3, 15, 16, 31, 40, 64])
def test_canonical_iupac_vs_oracle(k):
    rng = np.random.default_rng(400 + k)
    check_canonical(genome_with_rc_repeats(rng, [30_000, 9_000], b"ACGTACGTACGTNRYKMSWBDHV"), k)


def test_canonical_user_starts_gather_path():
    rng = np.random.default_rng(7)
    seqs = genome_with_rc_repeats(rng, [20_000], b"ACGT")
    sc = SequenceCollection(sequence_list=seqs)
    km = gk.Kmers(sc, min_kmer_len=25, max_kmer_len=25)
    user = rng.permutation(km.kmer_sba_start_indices)[:6000].astype(np.uint32)
    check_canonical(seqs, 25, user_starts=user)


def test_canonical_big_groups_and_palindromes():
    # poly-A / poly-T (each other's reverse complement) and a long palindromic run: groups far above
    # the local limit that tie on every key word
    seqs = [("a", "A" * 9000 + "T" * 9000), ("b", "ACGT" * 2500), ("c", "GC" * 3000)]
    for k in (31, 63):
        check_canonical(seqs, k)


def test_canonical_argument_errors():
    sc = SequenceCollection(sequence_list=[("a", "ACGTACGTAC")])
    km = gk.Kmers(sc, min_kmer_len=3, max_kmer_len=5)
    with pytest.raises(ValueError, match="canonical k-mers need min_kmer_len == max_kmer_len"):
        km.sort(canonical=True)
    km = gk.Kmers(sc, min_kmer_len=4, max_kmer_len=4)
    km.sort(canonical=True)
    with pytest.raises(ValueError, match="canonical k-mers are grouped at kmer_len == 4 only"):
        km.get_kmer_count(3)
    km.sort()
    with pytest.raises(AssertionError, match="needs sort"):
        km.get_canonical_strands()
    assert km.get_kmer_count(3) == 7


@pytest.mark.parametrize("k", [15, 31, 63])
def test_canonical_split_n_runs_vs_oracle(k):
    """Canonical k-mers over a GRCh38-like sba (N runs): the ACGT/other split keeps each k-mer's
    class under reverse complement, so it serves canonical sorts too."""
    rng = np.random.default_rng(600 + k)
    seqs = genome_with_rc_repeats(rng, [50_000, 20_000], b"ACGT")
    out = []
    for name, s in seqs:
        b = bytearray(s.encode())
        for a in rng.integers(0, len(b) - 300, 4):
            b[a:a + 200] = b"N" * 200
        b[int(rng.integers(0, len(b)))] = ord("R")
        out.append((name, b.decode()))
    km, _ = check_canonical(out, k)
    assert not km._engine.is_acgt()


@pytest.mark.parametrize("k", [15, 31])
def test_canonical_split_complementary_homopolymer_runs(k):
    """R runs and Y runs (complements) and self-complementary N / S runs: canonical R^k and Y^k are
    one k-mer, so their homopolymer groups merge in start order across both letters."""
    rng = np.random.default_rng(700 + k)
    seqs = genome_with_rc_repeats(rng, [40_000, 20_000], b"ACGT")
    out = []
    for name, s in seqs:
        b = bytearray(s.encode())
        for letter in b"RYNSMK":
            for a in rng.integers(100, len(b) - 400, 2):
                n_run = int(rng.integers(k + 1, k + 200))
                b[a:a + n_run] = bytes([letter]) * n_run
        out.append((name, b.decode()))
    km, _ = check_canonical(out, k)
    assert not km._engine.is_acgt()


# canonical 2-bit keys with a 64-bit first word (k >= 32) take an 8-bit L0, then packed pairs and
# a compact level where the bucket sizes call for them (C5); GKM_TEST_PAIRS=1 writes pairs wherever
# the bits fit, so these sizes run the pair and compact levels with their canonical tie phases
@pytest.mark.parametrize("k", [32, 63])
def test_canonical_pair_levels_vs_oracle(k, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_TEST_PAIRS", "1")
    rng = np.random.default_rng(500 + k)
    mixed = [("m" + name, s) for name, s in genome_with_rc_repeats(rng, [200_000], b"ACGT")]
    check_canonical(genome_with_rc_repeats(rng, [900_000, 300_000], b"AC") + mixed, k)
