"""The reference's own profiled sort workload (tools/run_profiling.py:226-236, profiling.py:367-448)
at test size: get_random_seq_list(1e6, 10) after np.random.seed(42), Kmers(min_kmer_len=1,
max_kmer_len=M).sort() for M = 20 (bounded variable length: LSD onesweep over (padded, length)
keys) and M = None (the Kmers default, suffix order: prefix doubling), bit-exact against the
oracle's break_ties=True order, and in the reference's default quicksort order on request.
bench.py --config ref_profile times the same workload at 1e8 bases."""

import sys
from pathlib import Path

import numpy as np
import pytest

from genome_kmers import _native
from genome_kmers import kmers as gk
from genome_kmers.sequence_collection import SequenceCollection
from oracle import oracle

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from bench import ref_profile_sba  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def workload():
    assert _native.device_count() > 0, "gpu tests need a visible MI355X"
    sba, seg = ref_profile_sba(1_000_000)
    parts = bytes(sba).split(b"$")
    sc = SequenceCollection(sequence_list=[(f"chr{i}", p.decode()) for i, p in enumerate(parts)])
    np.testing.assert_array_equal(sc.forward_sba, sba)
    return sc


@pytest.mark.parametrize("max_k", [20, None])
def test_ref_profile_sort_vs_oracle(workload, max_k):
    km = gk.Kmers(workload, min_kmer_len=1, max_kmer_len=max_k)
    unsorted = km.kmer_sba_start_indices.copy()
    assert len(unsorted) == 1_000_000
    km.sort()
    want = oracle.quicksort(workload.forward_sba, unsorted, 1, max_k, break_ties=True)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)
    kl = 20 if max_k else 12
    h, t = km.get_kmer_group_counts(kl, max_counts_bin=32)
    oh, ot = oracle.group_scan(workload.forward_sba, want, kl, max_counts_bin=32)
    np.testing.assert_array_equal(h, oh)
    assert t == ot


def test_ref_profile_reference_order(workload):
    km = gk.Kmers(workload, min_kmer_len=1, max_kmer_len=20)
    unsorted = km.kmer_sba_start_indices.copy()
    km.sort(order="reference")
    want = oracle.quicksort(workload.forward_sba, unsorted, 1, 20, break_ties=False)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)
