"""The C3 genome is the reference's own profiling genome (profiling.get_random_seq after
np.random.seed(seed), profiling.py:12-24): libgkm's host MT19937 (gk_reference_random_bases)
against numpy's legacy RandomState, which the reference draws from (np.random.choice over
["A", "T", "G", "C"] -> randint(0, 4)).  CPU only."""

import numpy as np
import pytest

from genome_kmers import _native, synthetic


def reference_get_random_seq(n, seed):
    # profiling.get_random_seq restated: np.random.seed + np.random.choice of the four letters
    np.random.seed(seed)
    bases = np.array(["A", "T", "G", "C"], dtype="U1")
    return "".join(np.random.choice(bases, n, replace=True)).encode()


@pytest.mark.parametrize("n,seed", [(0, 42), (1, 42), (623, 1), (624, 2), (625, 3), (10_000, 42), (100_003, 7)])
def test_matches_reference_generator(n, seed):
    assert _native.reference_random_bases(n, seed).tobytes() == reference_get_random_seq(n, seed)


def test_long_stream_and_c3_prefix():
    n = 3_000_000
    rs = np.random.RandomState(42)
    want = np.frombuffer(b"ATGC", dtype=np.uint8)[np.concatenate([rs.randint(0, 4, 1_000_001),
                                                                  rs.randint(0, 4, n - 1_000_001)])]
    sba, seg = synthetic.c3_genome(n, 42)
    np.testing.assert_array_equal(sba, want)
    assert seg.tolist() == [0]
