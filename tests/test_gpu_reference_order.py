"""Kmers.sort(order="reference"): the reference's DEFAULT tie order (numba quicksort with
break_ties=False, kmers.py:1624-1652), produced by libgkm (GK_SORT_QUICKSORT_ORDER: device sort,
then numba's quicksort on the host comparing the device's group ranks, gkm_qsort.cpp).

Pinned by the reference itself: ``starts_default`` and ``results_default_order`` of every golden
case (tests/golden/manifest.json, written by running the reference), including the queries that
name member locations (yield_first_n, kmer_info_to_yield="full"), which the stable order cannot
match inside tie groups.  At larger sizes: the oracle's restatement of the same quicksort.
"""

import numpy as np
import pytest

from conftest import load_manifest
from genome_kmers import _native, synthetic
from genome_kmers import kmers as gk
from genome_kmers.sequence_collection import SequenceCollection
from oracle import oracle
from test_gpu_parity import make, run_query

pytestmark = pytest.mark.gpu

CASES = load_manifest()


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert _native.device_count() > 0, "gpu tests need a visible MI355X"


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_reference_order_golden(case):
    km, a = make(case)
    km.sort(order="reference")
    np.testing.assert_array_equal(km.kmer_sba_start_indices, a["starts_default"])
    for q, want in zip(case["queries"], case["results_default_order"]):
        assert run_query(km, q) == want, q


def test_reference_order_user_starts_keeps_their_initial_order():
    # the quicksort starts from the caller's order: a shuffled assignment sorts like the oracle's
    # quicksort of that same shuffled array
    rng = np.random.default_rng(9)
    unit = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 400).astype(np.uint8)
    s = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 20_000).astype(np.uint8)
    for at in (100, 5_000, 9_000, 15_000):
        s[at:at + 400] = unit
    sc = SequenceCollection(sequence_list=[("a", s.tobytes().decode())])
    km = gk.Kmers(sc, min_kmer_len=12, max_kmer_len=12)
    shuffled = rng.permutation(km.kmer_sba_start_indices).astype(np.uint32)
    km.kmer_sba_start_indices = shuffled.copy()
    km.sort(order="reference")
    want = oracle.quicksort(sc.forward_sba, shuffled, 12, 12, break_ties=False)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)


@pytest.mark.parametrize("min_k,max_k", [(31, 31), (5, 20), (3, None)])
def test_reference_order_c2_surrogate_vs_oracle(min_k, max_k):
    sba, _ = synthetic.c2_surrogate()
    L = 600_000 if max_k is None else len(sba)  # the unbounded oracle is slower per comparison
    sc = SequenceCollection(sequence_list=[("c2", bytes(sba[:L]).decode())])
    km = gk.Kmers(sc, min_kmer_len=min_k, max_kmer_len=max_k)
    unsorted = km.kmer_sba_start_indices.copy()
    km.sort(order="reference")
    want = oracle.quicksort(sc.forward_sba, unsorted, min_k, max_k, break_ties=False)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)
    # keys and counts are those of the stable order (only tie members moved)
    h, t = km.get_kmer_group_counts(max_k or min_k, max_counts_bin=64)
    oh, ot = oracle.group_scan(sc.forward_sba, want, max_k or min_k, max_counts_bin=64)
    np.testing.assert_array_equal(h, oh)
    assert t == ot


def test_reference_order_rejects_canonical():
    sc = SequenceCollection(sequence_list=[("a", "ACGTACGTAC" * 10)])
    km = gk.Kmers(sc, min_kmer_len=5, max_kmer_len=5)
    with pytest.raises(ValueError, match="canonical"):
        km.sort(canonical=True, order="reference")
    with pytest.raises(ValueError, match="order must be"):
        km.sort(order="quick")
