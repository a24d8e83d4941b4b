"""Parity at BASELINE.json's config scale on one GPU.

* C2 (E. coli K-12 surrogate, 4,641,652 bp, k = 31): bit-exact against the CPU oracle -- sorted
  starts vs the reference's quicksort in break_ties=True order (kmers.py:1624-1731, 1710-1711),
  group-size histogram, unique counts and encoded keys.
* C3 (3.1 Gb, k = 31), C4 (GRCh38-shaped, 24 contigs, N runs, k = 31) and C5 (the same, canonical
  k = 63) at FULL size: the oracle cannot sort 3.1e9 k-mers, so the output is checked on the
  device through size-independent properties (tests/devcheck.py: recomputed keys non-decreasing,
  ties in start order, a permutation of the enumerated starts, the product's keys, group sizes vs
  the product's group pass), plus oracle-checked windows of the sorted order at sorted indices on
  both sides of 2^31.
* The multi-chunk branches of the column scans and tile tables (which only full-size inputs reach
  with the production chunk sizes) re-run on the small parity inputs with test-only chunk sizes.
"""

import time

import numpy as np
import pytest

from genome_kmers import _native
from genome_kmers import kmers as gk
from genome_kmers import synthetic
from genome_kmers.sequence_collection import SequenceCollection
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if _native.device_count() == 0:
        pytest.skip("no GPU")


def _collection(sba, seg):
    """A SequenceCollection over an existing sba (the reference's attribute layout,
    sequence_collection.py:663-726) without re-joining 3.1e9 bytes through Python strings."""
    sc = SequenceCollection()
    sc.forward_sba = sba
    sc._forward_sba_seg_starts = np.asarray(seg, dtype=np.uint32)
    sc.forward_record_names = [f"chr{i}" for i in range(len(seg))]
    sc._strands_loaded = "forward"
    return sc


def _log(msg):
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


# ---------------------------------------------------------------------------------------------
# C2: bit-exact
# ---------------------------------------------------------------------------------------------
def test_c2_surrogate_bit_exact_vs_oracle():
    sba, seg = synthetic.c2_surrogate()
    assert sba.size == synthetic.C2_LENGTH
    sc = _collection(sba, seg)
    km = gk.Kmers(sc, min_kmer_len=31, max_kmer_len=31)
    n = synthetic.C2_LENGTH - 30
    assert len(km.kmer_sba_start_indices) == n == 4_641_622
    km.sort()
    got = km.kmer_sba_start_indices
    want = oracle.quicksort(sba, np.arange(n, dtype=np.uint32), 31, 31, break_ties=True)
    np.testing.assert_array_equal(got, want)
    h, t = km.get_kmer_group_counts(31, max_counts_bin=64)
    oh, ot = oracle.group_scan(sba, want, 31, max_counts_bin=64)
    np.testing.assert_array_equal(h, oh)
    assert t == ot == n
    assert h[7:].sum() > 0, "the planted 7-copy operons must give groups of size >= 7"
    first, counts = km.get_unique_kmers()
    assert int(counts.sum()) == n and len(first) == int(oh.sum())
    np.testing.assert_array_equal(np.bincount(np.minimum(counts, 64), minlength=65), oh)
    keys = km.get_encoded_kmers()
    np.testing.assert_array_equal(keys, oracle.encode_keys(sba, want, 2, 31, 0, 1))


# ---------------------------------------------------------------------------------------------
# C3 / C4 / C5 at full size
# ---------------------------------------------------------------------------------------------
def _full_size_check(sba, seg, k, canonical, product_keys, expect_n):
    import devcheck

    sc = _collection(sba, seg)
    t0 = time.time()
    km = gk.Kmers(sc, min_kmer_len=k, max_kmer_len=k)
    km.sort(canonical=canonical) if canonical else km.sort()
    eng = km._engine
    eng.sync()
    n = eng.n
    assert n == expect_n
    _log(f"sorted {n:,} {k}-mers in {time.time() - t0:.1f} s (incl. H2D)")
    hist_dev, total = km.get_kmer_group_counts(k, max_counts_bin=64)
    n_unique = eng.unique_count_only()  # group starts + multiplicities, resident in HBM
    gs_ptr, cnt_ptr, n_unique2 = eng.device_unique()
    assert total == n and n_unique2 == n_unique
    bits = 2 if eng.is_acgt() else 4
    if product_keys:
        starts_ptr, keys_ptr, n2, words = eng.device_views()
    else:
        starts_ptr, n2 = eng.device_starts()
    assert n2 == n
    chk = devcheck.SortedOutputCheck(sba, k, bits, canonical=canonical)
    # multi-word keys (C5: 4 words, 99 GB of product keys): recomputed one word at a time
    check = chk.check_sorted_wordwise if chk.words > 1 else chk.check_sorted
    groups, hist = check(starts_ptr, n, keys_ptr=keys_ptr if product_keys else 0,
                         key_words=words if product_keys else 0, max_counts_bin=64,
                         unique=(gs_ptr, cnt_ptr, n_unique))
    del chk
    _log(f"device property checks done ({time.time() - t0:.1f} s): {groups:,} groups")
    assert groups == n_unique
    np.testing.assert_array_equal(hist, hist_dev)
    offs = [0, 2**31 - 2048, 2**31 + 1, (2**31 + n) // 2, n - 4096]
    rng = np.random.default_rng(k)
    offs += list(rng.integers(0, n, 3))
    devcheck.oracle_windows(km, sba, k, offs, width=4096, canonical=canonical)
    _log(f"oracle windows done ({time.time() - t0:.1f} s)")
    return km


@pytest.mark.timeout(900)
def test_c3_full_size_properties():
    _log("C3: generating 3.1 Gb")
    sba, seg = synthetic.c3_genome()
    _full_size_check(sba, seg, 31, False, True, 3_099_999_970)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("k,canonical", [(31, False), (63, True)], ids=["c4_k31", "c5_k63_canonical"])
def test_grch38_surrogate_full_size_properties(k, canonical):
    # canonical k = 63: the product's own keys -- the 4-bit words the split sort's merge writes
    # from the packed sequence (the default path) -- against keys recomputed one word at a time
    # (devcheck.check_sorted_wordwise: 25 GB per word beside the product's 99 GB)
    _log("GRCh38 surrogate: generating")
    sba, seg = synthetic.grch38_surrogate(2)
    assert len(seg) == 24
    expect = sum(max(0, n - k + 1) for n in synthetic.GRCH38_LENGTHS)
    _full_size_check(sba, seg, k, canonical, True, expect)


@pytest.mark.timeout(900)
def test_c5_full_size_merge_keys_windows():
    """C5 at full size: the canonical 63-mer keys the split sort's merge writes from the packed
    sequence (gkm_split.hip put_key4_packed), read back in windows of the sorted order across the
    whole array (both ends, past 2^31, random offsets) and compared with the oracle's keys of the
    window's starts; the order inside every window is checked too."""
    import devcheck

    _log("GRCh38 surrogate: generating")
    sba, seg = synthetic.grch38_surrogate(2)
    sc = _collection(sba, seg)
    km = gk.Kmers(sc, min_kmer_len=63, max_kmer_len=63)
    km.sort(canonical=True)
    n = km._engine.n
    offs = [0, 2**31 - 2048, 2**31 + 1, n // 3, (2**31 + n) // 2, n - 4096]
    offs += list(np.random.default_rng(63).integers(0, n, 4))
    devcheck.oracle_windows(km, sba, 63, offs, width=4096, canonical=True, keys=True)
    _log("C5 merge-key windows done")


# ---------------------------------------------------------------------------------------------
# multi-chunk scan branches at parity-test sizes (test-only chunk sizes)
# ---------------------------------------------------------------------------------------------
@pytest.fixture
def small_chunks(monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_TEST_CHUNK_TILES", "2")
    monkeypatch.setitem(_native.options, "GKM_TEST_SCAN_CHUNK", "1024")


def _oracle_sorted(seqs, k, canonical=False):
    sc = SequenceCollection(sequence_list=seqs)
    km = gk.Kmers(sc, min_kmer_len=k, max_kmer_len=k)
    unsorted = km.kmer_sba_start_indices.copy()
    km.sort(canonical=canonical) if canonical else km.sort()
    if canonical:
        want = oracle.canonical_sort(sc.forward_sba, unsorted, k)
        oh, ot = oracle.canonical_group_hist(sc.forward_sba, want, k, max_counts_bin=32)
    else:
        want = oracle.quicksort(sc.forward_sba, unsorted, k, k, break_ties=True)
        oh, ot = oracle.group_scan(sc.forward_sba, want, k, max_counts_bin=32)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)
    h, t = km.get_kmer_group_counts(k, max_counts_bin=32)
    np.testing.assert_array_equal(h, oh)
    assert t == ot
    first, counts = km.get_unique_kmers()
    assert int(counts.sum()) == len(want)
    return km


def _genome(seed, lengths, alphabet=b"ACGT", rep_len=3000, copies=12, n_runs=0):
    rng = np.random.default_rng(seed)
    rep = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), rep_len).astype(np.uint8)
    seqs = []
    for i, L in enumerate(lengths):
        s = rng.choice(np.frombuffer(alphabet, dtype=np.uint8), L).astype(np.uint8)
        for _ in range(copies):
            at = int(rng.integers(0, L - rep_len))
            s[at:at + rep_len] = rep
        for _ in range(n_runs):
            at = int(rng.integers(0, L - 500))
            s[at:at + int(rng.integers(40, 500))] = ord("N")
        seqs.append((f"c{i}", s.tobytes().decode()))
    return seqs


@pytest.mark.parametrize("k", [21, 31])
def test_small_chunks_acgt_vs_oracle(small_chunks, k):
    # ~1.2 M k-mers: L0 buckets of ~9 k keys span several 11,264-key tiles -> several 2-tile
    # chunks per bucket at L1; the selection scans have > 1024 tiles
    _oracle_sorted(_genome(5, [900_000, 300_000]), k)


@pytest.mark.parametrize("fused_uniform", [True, False])
def test_small_chunks_low_entropy_levels_vs_oracle(small_chunks, monkeypatch, fused_uniform):
    # deep levels: the uniform-bucket drop behind the classify's read-back (default) or its own
    if not fused_uniform:
        monkeypatch.setitem(_native.options, "GKM_NO_FUSED_UNIFORM", "1")
    monkeypatch.setitem(_native.options, "GKM_LEVEL_BITS", "8,6")
    _oracle_sorted(_genome(6, [600_000], alphabet=b"AACGTT", rep_len=5000, copies=20), 31)


@pytest.mark.parametrize("fused_uniform", [True, False])
def test_deep_levels_identical_repeats_vs_oracle(monkeypatch, fused_uniform):
    # buckets of > 8,192 copies of one k-mer (uniform: dropped) beside near-identical ones (another
    # level each) several levels down -- the deep levels of a repeat-rich genome
    if not fused_uniform:
        monkeypatch.setitem(_native.options, "GKM_NO_FUSED_UNIFORM", "1")
    rng = np.random.default_rng(11)
    s = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 1_500_000).astype(np.uint8)
    s[100_000:140_000] = np.frombuffer(b"CA" * 20_000, dtype=np.uint8)  # (CA)n: two uniform buckets
    unit = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 60).astype(np.uint8)
    for j in range(9000):  # 9,000 copies of a 60-mer, one substitution each at a late position
        u = unit.copy()
        u[40 + j % 20] = b"ACGT"[(j // 20) % 4]
        s[200_000 + 61 * j:200_000 + 61 * j + 60] = u
    _oracle_sorted([("c0", s.tobytes().decode())], 31)


@pytest.mark.parametrize("k", [21, 31])
def test_level_bucket_scan_multi_launch_vs_oracle(small_chunks, monkeypatch, k):
    # the level tables' bucket scans as seg_counts + two device-wide scans (the branch for more
    # than 65,536 big buckets, which no parity-size input reaches), totals cross-checked
    monkeypatch.setitem(_native.options, "GKM_TEST_SEG_SCAN_MULTI", "1")
    _oracle_sorted(_genome(5, [900_000, 300_000]), k)
    _oracle_sorted(_genome(6, [600_000], alphabet=b"AACGTT", rep_len=5000, copies=20), k)


@pytest.mark.parametrize("chunk_mb", ["0", "2", "6"])
def test_mapped_buffers_vs_oracle(monkeypatch, chunk_mb):
    # the k-mer arrays and scratch as address ranges mapped from 2 / 6 MiB physical allocations
    # (many chunks per array, buffers regrown between the sorts), or plain hipMalloc ("0")
    monkeypatch.setitem(_native.options, "GKM_VMM_CHUNK_MB", chunk_mb)
    monkeypatch.setitem(_native.options, "GKM_TEST_VMM_MIN_KB", "64")
    _oracle_sorted(_genome(12, [700_000, 200_000], n_runs=5), 31)
    _oracle_sorted(_genome(13, [2_500_000]), 31)
    _oracle_sorted(_genome(14, [600_000], n_runs=5), 63, canonical=True)


@pytest.mark.parametrize("k", [31, 63])
def test_small_chunks_split_n_runs_vs_oracle(small_chunks, k):
    _oracle_sorted(_genome(7, [500_000, 400_000], n_runs=40), k)


@pytest.mark.parametrize("k", [31, 63])
def test_small_chunks_canonical_vs_oracle(small_chunks, k):
    _oracle_sorted(_genome(8, [700_000], n_runs=10), k, canonical=True)


def test_small_chunks_key_ranges_concatenate(small_chunks):
    from genome_kmers import distributed as D

    seqs = _genome(9, [800_000, 200_000])
    sc = SequenceCollection(sequence_list=seqs)
    sba, seg = sc.forward_sba, sc._forward_sba_seg_starts
    km = gk.Kmers(sc, min_kmer_len=31, max_kmer_len=31)
    km.sort()
    want = km.kmer_sba_start_indices.copy()
    e = _native.Engine()
    e.set_sequence(sba, seg)
    world = 3
    pos = D.position_ranges(len(sba), world)
    H = None
    for r in range(world):
        h, _bits = e.shard_histogram(pos[r], pos[r + 1], 31)
        H = h.astype(np.int64) if H is None else H + h.astype(np.int64)
    cuts = D.split_buckets(H, world)
    parts = []
    for r in range(world):
        e.shard_sort_range(31, cuts[r], cuts[r + 1])
        parts.append(e.copy_starts())
    np.testing.assert_array_equal(np.concatenate(parts), want)


# ---------------------------------------------------------------------------------------------
# multi-word keys of a sorted enumeration through the position-indexed 2-bit row table
# (gkm_encode.hip key_rows2_kernel / row2_gather_kernel): every row dispatch (2-bit W 2; 4-bit
# W 2, 3, 4), canonical and forward, windows with N runs / IUPAC letters (marker rows), several
# contigs (rows across the '$' separators) and a contig shorter than 16 positions
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("k,alphabet,canonical", [
    (33, b"ACGT", False), (63, b"ACGT", True), (40, b"ACGTACGTACGTRYKMSWBDHV", False),
    (48, b"ACGTACGTACGTACGTN", True), (63, b"ACGTACGTACGTACGTACGTN", True), (63, b"ACGTACGTACGTNRY", False),
    (24, b"ACGTACGTACGTACGTACGTRY", True)])
def test_key_rows_vs_oracle(k, alphabet, canonical):
    seqs = _genome(50 + k, [60_000, 25_000], alphabet=alphabet, rep_len=2000, copies=4, n_runs=3)
    seqs.append(("tiny", "ACGTTGCA" * 9 + "AC"))  # 74 bases: k-mers near a contig end
    sc = SequenceCollection(sequence_list=seqs)
    km = gk.Kmers(sc, min_kmer_len=k, max_kmer_len=k)
    unsorted = km.kmer_sba_start_indices.copy()
    km.sort(canonical=canonical) if canonical else km.sort()
    words, bits, _ = km._engine.key_layout()
    if canonical:
        want = oracle.canonical_sort(sc.forward_sba, unsorted, k)
        want_keys = oracle.canonical_keys(sc.forward_sba, want, k, bits)
    else:
        want = oracle.quicksort(sc.forward_sba, unsorted, k, k, break_ties=True)
        spec = oracle.key_spec(km._engine.is_acgt(), k, k)
        want_keys = oracle.encode_keys(sc.forward_sba, want, *spec)
    np.testing.assert_array_equal(km.kmer_sba_start_indices, want)
    np.testing.assert_array_equal(km.get_encoded_kmers(), want_keys)
