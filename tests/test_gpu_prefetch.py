"""The sort hint (gk_sort_hint): gk_set_sequence runs the L0 pass of gk_sort(k) over regions of a
A/C/G/T sequence (one or many contigs) while the packed transfer lands them, and the next gk_sort(k) of the
whole enumeration starts from the regions' buckets (gkm_msd.hip, L0Prefetch).

The result must be bit-identical to the sort without the hint -- sorted starts, keys, head flags
(through the unique counts) -- and to the oracle's break_ties=True order; the tests also check that
the prefetched pass was the one used (profile stages), and that every other use of the k-mer
buffers, another k, canonical sorts and user-given starts fall back to the plain sort; on a mixed sba
(N runs, IUPAC letters) the prefetched pass is the class-A L0 of the split sort.  Small chunk and region sizes (GKM_PACK_BLOCKS, GKM_PREFETCH_REGIONS) put
many regions, partial tiles and region edges into test-sized inputs."""

import numpy as np
import pytest

from genome_kmers import _native
from genome_kmers.kmers import Kmers
from genome_kmers.sequence_collection import SequenceCollection
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert _native.device_count() > 0, "gpu tests need a visible MI355X"


def genome(rng, L, repeat=0, copies=0):
    s = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, L)].copy()
    if repeat:
        rep = s[:repeat].copy()
        for at in rng.integers(0, L - repeat, copies):
            s[at:at + repeat] = rep
    return s


def product(eng, k):
    n = eng.enumerate(k)
    eng.sort(k)
    starts = eng.copy_starts(np.empty(n, dtype=np.uint32))
    keys = eng.copy_keys()
    first, counts = eng.unique_counts()
    return starts, keys, first, counts


def run(sba, seg, k, monkeypatch, hint, regions=7, blocks=1, threads=3):
    monkeypatch.setenv("GKM_PACK_MIN", "0")
    monkeypatch.setenv("GKM_PACK_BLOCKS", str(blocks))
    monkeypatch.setenv("GKM_XFER_THREADS", str(threads))
    monkeypatch.setenv("GKM_PREFETCH_REGIONS", str(regions))
    eng = _native.Engine()
    eng.profile_enable(True)
    if hint:
        eng.sort_hint(k)
    eng.set_sequence(sba, seg)
    out = product(eng, k)
    rep = eng.profile_report()
    eng.profile_enable(False)
    for v in ("GKM_PACK_MIN", "GKM_PACK_BLOCKS", "GKM_XFER_THREADS", "GKM_PREFETCH_REGIONS"):
        monkeypatch.delenv(v)
    return eng, out, rep


def same(a, b):
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("k", [8, 15, 31, 32])
@pytest.mark.parametrize("L,regions", [(70_001, 1), (300_000, 7), (1_000_003, 16)])
def test_prefetched_sort_matches_plain(k, L, regions, monkeypatch):
    rng = np.random.default_rng(L + k)
    sba = genome(rng, L, repeat=700, copies=5)
    seg = np.zeros(1, dtype=np.uint32)
    _, got, rep = run(sba, seg, k, monkeypatch, True, regions)
    assert "prefetch_l0" in rep and "msd_pass_l0" not in rep, sorted(rep)
    _, want, rep0 = run(sba, seg, k, monkeypatch, False, regions)
    assert "prefetch_l0" not in rep0 and "msd_pass_l0" in rep0
    same(got, want)
    if L <= 300_000:
        ref = oracle.quicksort(sba, np.arange(L - k + 1, dtype=np.uint32), k, k, break_ties=True)
        np.testing.assert_array_equal(got[0], ref)


@pytest.mark.parametrize("mode", ["p88", "p88_pairs"])
@pytest.mark.parametrize("alphabet", [b"ACGT", b"AC"])
def test_prefetch_packed_l0(mode, alphabet, monkeypatch):
    # the regions write the packed L0 form (GKM_TEST_P88=1); the first level from their pieces reads
    # it when it writes packed pairs (GKM_TEST_PAIRS=1), else the pieces are expanded first
    monkeypatch.setitem(_native.options, "GKM_TEST_P88", "1")
    if mode == "p88_pairs":
        monkeypatch.setitem(_native.options, "GKM_TEST_PAIRS", "1")
    rng = np.random.default_rng(len(alphabet) + len(mode))
    L = 900_000
    sba = np.frombuffer(alphabet, dtype=np.uint8)[rng.integers(0, len(alphabet), L)].copy()
    seg = np.zeros(1, dtype=np.uint32)
    _, got, rep = run(sba, seg, 31, monkeypatch, True, regions=9)
    assert "prefetch_l0" in rep and "msd_pass_l0" not in rep
    _, want, _ = run(sba, seg, 31, monkeypatch, False, regions=9)
    same(got, want)
    np.testing.assert_array_equal(got[0], oracle.quicksort(sba, np.arange(L - 30, dtype=np.uint32), 31, 31,
                                                           break_ties=True))


def test_prefetch_many_chunks_threads_and_regions(monkeypatch):
    # chunks finish out of order on 8 packing threads; 40 regions of one tile each, the last partial
    rng = np.random.default_rng(9)
    L = 40 * 24576 - 5000
    sba = genome(rng, L, repeat=3000, copies=9)
    seg = np.zeros(1, dtype=np.uint32)
    _, got, rep = run(sba, seg, 31, monkeypatch, True, regions=40, blocks=1, threads=8)
    assert rep["prefetch_l0"]["units"] == L - 30
    _, want, _ = run(sba, seg, 31, monkeypatch, False)
    same(got, want)


@pytest.mark.parametrize("chunk_tiles", ["1", "2", "3"])
def test_prefetch_multi_chunk_region_scans(chunk_tiles, monkeypatch):
    # regions of 5 tiles in column-scan chunks of 1-3 tiles, the last region shorter (fewer chunks
    # than the others: its tables sit at the same stride) -- the multi-chunk scan branch that only
    # full-size inputs reach with the default 256-tile chunks
    monkeypatch.setitem(_native.options, "GKM_TEST_CHUNK_TILES", chunk_tiles)
    rng = np.random.default_rng(int(chunk_tiles))
    L = 32 * 24576 + 1234
    sba = genome(rng, L, repeat=2000, copies=7)
    seg = np.zeros(1, dtype=np.uint32)
    _, got, rep = run(sba, seg, 31, monkeypatch, True, regions=7)
    assert "prefetch_l0" in rep and "msd_pass_l0" not in rep
    monkeypatch.delitem(_native.options, "GKM_TEST_CHUNK_TILES")
    _, want, _ = run(sba, seg, 31, monkeypatch, False)
    same(got, want)
    np.testing.assert_array_equal(got[0], oracle.quicksort(sba, np.arange(L - 30, dtype=np.uint32), 31, 31,
                                                           break_ties=True))


def test_prefetch_large_packed_pair_levels():
    # 3e8 bases: the first level from the prefetched pieces writes packed pairs and the compact level
    # behind it reads them (the C3 level structure), with the default chunking and 16 regions
    from genome_kmers import synthetic

    sba, seg = synthetic.c3_genome(300_000_000, 42)
    outs = []
    for hint in (31, 0):
        eng = _native.Engine()
        eng.sort_hint(hint)
        eng.profile_enable(True)
        eng.set_sequence(sba, seg)
        n = eng.enumerate(31)
        eng.sort(31)
        rep = eng.profile_report()
        assert ("prefetch_l0" in rep) == (hint != 0) and ("msd_pass_l1p" in rep or "msd_pass_l1" in rep)
        outs.append(eng.copy_starts(np.empty(n, dtype=np.uint32)))
        del eng
    np.testing.assert_array_equal(outs[0], outs[1])


def test_prefetch_consumed_once_and_dropped_by_other_calls(monkeypatch):
    rng = np.random.default_rng(4)
    L = 200_000
    sba = genome(rng, L, repeat=500, copies=4)
    seg = np.zeros(1, dtype=np.uint32)
    eng, got, _ = run(sba, seg, 21, monkeypatch, True, regions=5)
    _, want, _ = run(sba, seg, 21, monkeypatch, False)
    same(got, want)
    # the second sort of the same engine: no prefetched pass left, the plain L0 runs
    eng.profile_enable(True)
    again = product(eng, 21)
    rep = eng.profile_report()
    eng.profile_enable(False)
    assert "msd_pass_l0" in rep and "prefetch_l0" not in rep
    same(again, want)
    ref = oracle.quicksort(sba, np.arange(L - 20, dtype=np.uint32), 21, 21, break_ties=True)
    # another k after a hinted transfer: plain path, correct
    monkeypatch.setenv("GKM_PACK_MIN", "0")
    monkeypatch.setenv("GKM_PACK_BLOCKS", "1")
    for other in ("k", "starts", "canonical", "max"):
        e2 = _native.Engine()
        e2.sort_hint(21)
        e2.set_sequence(sba, seg)
        if other == "k":
            n = e2.enumerate(17)
            e2.sort(17)
            np.testing.assert_array_equal(e2.copy_starts(np.empty(n, dtype=np.uint32)),
                                          oracle.quicksort(sba, np.arange(L - 16, dtype=np.uint32), 17, 17,
                                                           break_ties=True))
        elif other == "starts":
            user = rng.permutation(L - 20).astype(np.uint32)[:50_000]
            e2.set_start_indices(user, 21)
            e2.sort(21)
            np.testing.assert_array_equal(e2.copy_starts(np.empty(len(user), dtype=np.uint32)),
                                          oracle.quicksort(sba, np.sort(user), 21, 21, break_ties=True))
        elif other == "canonical":
            n = e2.enumerate(21)
            e2.sort(21, canonical=True)
            e3 = _native.Engine()
            e3.set_sequence(sba, seg)
            e3.enumerate(21)
            e3.sort(21, canonical=True)
            np.testing.assert_array_equal(e2.copy_starts(np.empty(n, dtype=np.uint32)),
                                          e3.copy_starts(np.empty(n, dtype=np.uint32)))
        else:  # a longer bound than the hint: not the prefetched spec
            n = e2.enumerate(21)
            e2.sort(25)
            np.testing.assert_array_equal(e2.copy_starts(np.empty(n, dtype=np.uint32)),
                                          oracle.quicksort(sba, np.arange(L - 20, dtype=np.uint32), 21, 25,
                                                           break_ties=True))
    monkeypatch.delenv("GKM_PACK_MIN")
    monkeypatch.delenv("GKM_PACK_BLOCKS")
    np.testing.assert_array_equal(got[0], ref)


def contigs(rng, lengths, repeat=0, copies=0):
    """'$'-joined random ACGT contigs (the reference's forward_sba layout) and their starts."""
    parts = [genome(rng, n, min(repeat, n // 2), copies) for n in lengths]
    seg = np.cumsum([0] + [n + 1 for n in lengths[:-1]]).astype(np.uint32)
    sba = np.concatenate([np.concatenate([p, np.frombuffer(b"$", dtype=np.uint8)]) for p in parts])[:-1]
    return np.ascontiguousarray(sba), seg


# Round 6: multi-contig ACGT sequences prefetch too (the '$' separators are stops of the region
# passes, their blocks cross the link raw); bit-identical to the plain sort and to the oracle
@pytest.mark.parametrize("k", [12, 31, 32])
@pytest.mark.parametrize("lengths,regions", [
    ([70_000, 80_000], 4),
    ([30_000 + 997 * i for i in range(24)], 9),             # 24 contigs: separators in many regions
    ([100, 40_000, 31, 32, 33, 90_000, 24_576, 12], 6),    # contigs of k bases, tile-sized ones
])
def test_prefetch_multi_contig(k, lengths, regions, monkeypatch):
    rng = np.random.default_rng(len(lengths) + k)
    # (the reference rejects min_kmer_len > the shortest sequence: the contigs shorter than k drop out)
    sba, seg = contigs(rng, [n for n in lengths if n >= k], repeat=600, copies=3)
    _, got, rep = run(sba, seg, k, monkeypatch, True, regions=regions)
    assert "prefetch_l0" in rep and "msd_pass_l0" not in rep, sorted(rep)
    _, want, rep0 = run(sba, seg, k, monkeypatch, False, regions=regions)
    assert "prefetch_l0" not in rep0
    same(got, want)
    np.testing.assert_array_equal(got[0], oracle.quicksort(sba, oracle.enumerate_starts(sba, seg, k), k, k,
                                                           break_ties=True))


# Round 6: a mixed sba (N runs, IUPAC letters) prefetches its class-A L0 (the region passes stop
# k-mers at every non-ACGT byte) and the split sort's A sort starts from it (gkm_split.hip)
@pytest.mark.parametrize("k", [16, 31])
@pytest.mark.parametrize("kind", ["N", "N_contigs", "iupac_late"])
def test_prefetch_mixed_alphabet(kind, k, monkeypatch):
    rng = np.random.default_rng(12)
    L = 150_000
    sba = genome(rng, L)
    seg = np.zeros(1, dtype=np.uint32)
    if kind == "N":
        sba[90_000:90_050] = ord("N")
    elif kind == "N_contigs":  # 24 contigs with N runs (the GRCh38 shape)
        sba, seg = contigs(rng, [6_000 + 50 * i for i in range(24)])
        for at in range(1_000, len(sba) - 200, 9_000):
            sba[at:at + 120] = ord("N")
    else:  # one IUPAC letter in the last chunk: regions before it have run, the prefetch is dropped
        sba[L - 40] = ord("R")
    _, got, rep = run(sba, seg, k, monkeypatch, True, regions=4)
    assert "prefetch_l0" in rep and "split_merge" in rep and "msd_pass_l0" not in rep, sorted(rep)
    _, want, rep0 = run(sba, seg, k, monkeypatch, False, regions=4)
    assert "prefetch_l0" not in rep0 and "split_merge" in rep0
    same(got, want)
    np.testing.assert_array_equal(got[0], oracle.quicksort(sba, oracle.enumerate_starts(sba, seg, k), k, k,
                                                           break_ties=True))


def test_kmers_api_fixed_length_uses_the_hint(monkeypatch):
    # the drop-in path: Kmers(sc, k, k) hints the transfer, sort() finishes from the prefetched pass
    monkeypatch.setenv("GKM_PACK_MIN", "0")
    monkeypatch.setenv("GKM_PACK_BLOCKS", "1")
    monkeypatch.setenv("GKM_PREFETCH_REGIONS", "6")
    rng = np.random.default_rng(21)
    s = genome(rng, 180_000, repeat=400, copies=6)
    sc = SequenceCollection(sequence_list=[("chr", s.tobytes().decode())])
    km = Kmers(sc, min_kmer_len=31, max_kmer_len=31)
    km.sort()
    want = oracle.quicksort(sc.forward_sba, np.arange(len(s) - 30, dtype=np.uint32), 31, 31, break_ties=True)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)
    hist, total = km.get_kmer_group_counts(31, max_counts_bin=16)
    ohist, ototal = oracle.group_scan(sc.forward_sba, want, 31, max_counts_bin=16)
    assert np.array_equal(hist, ohist) and total == ototal
