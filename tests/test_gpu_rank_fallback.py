"""The partitions' fallback ranking (gk_rank_mode, gkm_partition.h rank_ballot).

Every stable partition of the device sort ranks an item by one returning LDS atomic, which relies
on gfx950 applying same-address lanes in lane order; gk_create checks that per device and, where it
fails, switches every partition to a ballot-match ranking.  These tests force that fallback on the
device (it is never needed on a healthy MI355X) and rerun golden sort cases, the C2 surrogate and
multi-word / canonical / IUPAC cases: the order must stay bit-exact (reference break_ties=True
order, kmers.py:1654-1731; the oracle's restatement of it).
"""

import numpy as np
import pytest

from conftest import load_case, load_manifest, seq_list_of
from genome_kmers import _native, synthetic
from genome_kmers import kmers as gk
from genome_kmers.sequence_collection import SequenceCollection
from oracle import oracle

pytestmark = pytest.mark.gpu

CASES = load_manifest()


@pytest.fixture(scope="module", autouse=True)
def ballot_ranking():
    assert _native.device_count() > 0, "gpu tests need a visible MI355X"
    eng = _native.Engine()
    assert eng.rank_mode(1) == 1
    yield
    eng.rank_mode(0)
    assert _native.Engine().rank_mode() == 0, "the device's default ranking was not restored"


def test_mode_persists_across_contexts():
    assert _native.Engine().rank_mode() == 1


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_sort_golden_ballot_ranking(case):
    a = load_case(case["name"])
    sc = SequenceCollection(sequence_list=seq_list_of(case, a), strands_to_load="forward")
    km = gk.Kmers(sc, min_kmer_len=case["min_kmer_len"], max_kmer_len=case["max_kmer_len"])
    km.sort()
    np.testing.assert_array_equal(km.kmer_sba_start_indices, a["starts_stable"])


def _check(seqs, k, canonical=False):
    sc = SequenceCollection(sequence_list=seqs)
    eng = _native.Engine()
    eng.set_sequence(sc.forward_sba, sc._forward_sba_seg_starts)
    n = eng.enumerate(k)
    eng.sort(k, canonical=canonical)
    got = eng.copy_starts(np.empty(n, dtype=np.uint32))
    unsorted = oracle.enumerate_starts(sc.forward_sba, sc._forward_sba_seg_starts, k)
    if canonical:
        want = oracle.canonical_sort(sc.forward_sba, unsorted, k)
    else:
        want = oracle.quicksort(sc.forward_sba, unsorted, k, k, break_ties=True)
    np.testing.assert_array_equal(got, want)


def test_c2_surrogate_ballot_ranking():
    sba, seg = synthetic.c2_surrogate()
    seqs = [("c2", bytes(sba).decode())]
    _check(seqs, 31)


@pytest.mark.parametrize("alphabet,k,canonical", [(b"ACGT", 63, False), (b"ACGT", 40, True),
                                                   (b"ACGTACGTACGTNRY", 33, False), (b"ACGTN", 63, True)])
def test_multiword_ballot_ranking(alphabet, k, canonical):
    rng = np.random.default_rng(11)
    rep = rng.choice(np.frombuffer(alphabet, dtype=np.uint8), 3000).astype(np.uint8)
    seqs = []
    for i, L in enumerate([120_000, 60_000, 9_000]):
        s = rng.choice(np.frombuffer(alphabet, dtype=np.uint8), L).astype(np.uint8)
        for _ in range(5):
            at = int(rng.integers(0, L - len(rep)))
            s[at:at + len(rep)] = rep
        seqs.append((f"c{i}", s.tobytes().decode()))
    _check(seqs, k, canonical)


def test_user_starts_onesweep_ballot_ranking():
    # host-provided starts in random order: sorted by the LSD onesweep path (gkm_onesweep.h)
    rng = np.random.default_rng(5)
    seq = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 200_000).astype(np.uint8).tobytes().decode()
    sc = SequenceCollection(sequence_list=[("a", seq), ("b", seq[:50_000])])
    unsorted = oracle.enumerate_starts(sc.forward_sba, sc._forward_sba_seg_starts, 31)
    shuffled = rng.permutation(unsorted).astype(np.uint32)
    eng = _native.Engine()
    eng.set_sequence(sc.forward_sba, sc._forward_sba_seg_starts)
    eng.set_start_indices(shuffled, 31)
    eng.sort(31)
    want = oracle.quicksort(sc.forward_sba, unsorted, 31, 31, break_ties=True)
    np.testing.assert_array_equal(eng.copy_starts(), want)
