"""The packed sba transfer of gk_set_sequence (gkm_xfer.hip): 64 KiB blocks of pure A/C/G/T cross
the link as 2-bit codes, every other block raw, unpacked into the resident ASCII sba on the device;
the alphabet check (sequence_collection.py:441-458, 694-697) is taken on the host while packing.

Checked against the plain copy path on the same inputs: the resident bytes (read back), the
alphabet outcome (ACGT-only flag, non-allowed bytes -> the reference's error, '$' census) and the
sorted k-mers.  Small block-per-chunk counts and thread counts force many chunks and slot reuse
at test sizes (GKM_PACK_MIN=0, GKM_PACK_BLOCKS, GKM_XFER_THREADS)."""

import numpy as np
import pytest

from genome_kmers import _native
from oracle import oracle

pytestmark = pytest.mark.gpu

B = 64 * 1024


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert _native.device_count() > 0, "gpu tests need a visible MI355X"


def genome(rng, L, contigs=1, n_runs=0, iupac=0):
    s = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, L)].copy()
    for _ in range(n_runs):
        at = int(rng.integers(0, L - 5000))
        s[at:at + int(rng.integers(1, 5000))] = ord("N")
    for p in rng.integers(0, L, iupac):
        s[p] = np.frombuffer(b"RYSWKMBDHVN", dtype=np.uint8)[rng.integers(0, 11)]
    cuts = np.sort(rng.choice(np.arange(100, L - 100, 50), contigs - 1, replace=False)) if contigs > 1 else []
    for c in cuts:
        s[c] = ord("$")
    seg = np.concatenate([[0], np.asarray(cuts, dtype=np.int64) + 1]).astype(np.uint32)
    return s, seg


def load(sba, seg, monkeypatch, packed, blocks=2, threads=3):
    if packed:
        monkeypatch.setenv("GKM_PACK_MIN", "0")
        monkeypatch.setenv("GKM_PACK_BLOCKS", str(blocks))
        monkeypatch.setenv("GKM_XFER_THREADS", str(threads))
    else:
        monkeypatch.setenv("GKM_PACK_MIN", str(1 << 62))
    eng = _native.Engine()
    eng.set_sequence(sba, seg)
    for v in ("GKM_PACK_MIN", "GKM_PACK_BLOCKS", "GKM_XFER_THREADS"):
        monkeypatch.delenv(v, raising=False)
    return eng


CASES = [
    # (length, contigs, N runs, scattered IUPAC letters)
    (1, 1, 0, 0), (63, 1, 0, 0), (64, 1, 0, 0), (65, 1, 0, 0), (B - 1, 1, 0, 0), (B, 1, 0, 0),
    (B + 33, 1, 0, 0), (5 * B + 17, 1, 0, 0), (9 * B, 3, 0, 0), (700_001, 5, 2, 0), (1_000_003, 2, 0, 7),
    (2_000_000, 24, 6, 3),
]


@pytest.mark.parametrize("L,contigs,runs,iupac", CASES)
@pytest.mark.parametrize("blocks,threads", [(1, 1), (2, 3), (128, 16)])
def test_packed_transfer_matches_plain(L, contigs, runs, iupac, blocks, threads, monkeypatch):
    rng = np.random.default_rng(L + 7 * contigs + runs)
    sba, seg = genome(rng, max(L, 200) if contigs > 1 else L, contigs, runs, iupac)
    packed = load(sba, seg, monkeypatch, True, blocks, threads)
    np.testing.assert_array_equal(packed.copy_sequence(len(sba)), sba)
    plain = load(sba, seg, monkeypatch, False)
    assert packed.is_acgt() == plain.is_acgt() == (runs == 0 and iupac == 0)
    k = 11 if len(sba) > 11 * contigs else 1
    shortest = np.diff(np.concatenate([seg.astype(np.int64), [len(sba) + 1]])).min() - 1
    k = int(min(k, shortest))
    outs = []
    for eng in (packed, plain):
        n = eng.enumerate(k)
        eng.sort(k)
        outs.append(eng.copy_starts(np.empty(n, dtype=np.uint32)))
    np.testing.assert_array_equal(outs[0], outs[1])


def test_packed_transfer_sorts_like_the_oracle(monkeypatch):
    rng = np.random.default_rng(3)
    sba, seg = genome(rng, 3 * B + 999, contigs=3, n_runs=1, iupac=2)
    eng = load(sba, seg, monkeypatch, True, blocks=1, threads=2)
    n = eng.enumerate(31)
    eng.sort(31)
    want = oracle.quicksort(sba, oracle.enumerate_starts(sba, seg, 31), 31, 31, break_ties=True)
    np.testing.assert_array_equal(eng.copy_starts(np.empty(n, dtype=np.uint32)), want)


@pytest.mark.parametrize("bad", [ord("a"), ord("X"), 0, 255, ord("U")])
@pytest.mark.parametrize("where", [0, B - 1, B, 3 * B + 5])
def test_packed_transfer_rejects_bytes_outside_the_alphabet(bad, where, monkeypatch):
    rng = np.random.default_rng(where)
    sba, seg = genome(rng, 4 * B)
    sba[where] = bad
    for packed in (True, False):
        with pytest.raises(_native.GkError) as ei:
            load(sba, seg, monkeypatch, packed)
        assert ei.value.code == _native.GK_E_ALPHABET


def test_internal_dollar_detected_on_both_paths(monkeypatch):
    rng = np.random.default_rng(5)
    sba, seg = genome(rng, 3 * B)
    sba[B + 10] = ord("$")  # a '$' that is not a segment separator
    for packed in (True, False):
        eng = load(sba, seg, monkeypatch, packed)
        eng.enumerate(5)
        with pytest.raises(_native.GkError) as ei:
            eng.sort(5)
        assert ei.value.code == _native.GK_E_NO_BASES


def test_default_threshold_large_input():
    # 40 MB: above GKM_PACK_MIN's default, so the packed path with its default chunking runs
    rng = np.random.default_rng(11)
    sba = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, 40_000_001)]
    sba[12_345_678:12_350_000] = ord("N")
    eng = _native.Engine()
    eng.set_sequence(sba, np.zeros(1, dtype=np.uint32))
    np.testing.assert_array_equal(eng.copy_sequence(len(sba)), sba)
    assert not eng.is_acgt()


def pinned_copy(a):
    import torch

    t = torch.empty(len(a), dtype=torch.uint8).pin_memory()
    t.numpy()[:] = a
    return t  # keep the tensor alive: its numpy view is the pinned buffer


@pytest.mark.parametrize("runs,iupac", [(0, 0), (3, 5)])
@pytest.mark.parametrize("blocks,threads", [(1, 1), (2, 4)])
@pytest.mark.parametrize("hybrid", ["0", "1"])
def test_pinned_source_hybrid_transfer(runs, iupac, blocks, threads, hybrid, monkeypatch):
    # a pinned source; GKM_XFER_HYBRID=1: chunks go packed from the front and raw (DMA, device
    # census) from the back
    monkeypatch.setenv("GKM_XFER_HYBRID", hybrid)
    rng = np.random.default_rng(17 + runs)
    sba, seg = genome(rng, 40 * B + 1234, contigs=4, n_runs=runs, iupac=iupac)
    t = pinned_copy(sba)
    packed = load(t.numpy(), seg, monkeypatch, True, blocks, threads)
    np.testing.assert_array_equal(packed.copy_sequence(len(sba)), sba)
    plain = load(sba, seg, monkeypatch, False)
    assert packed.is_acgt() == plain.is_acgt()
    outs = []
    for eng in (packed, plain):
        n = eng.enumerate(15)
        eng.sort(15)
        outs.append(eng.copy_starts(np.empty(n, dtype=np.uint32)))
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("where", [0, 20 * B + 3, 40 * B - 1])
def test_pinned_source_rejects_bad_bytes_anywhere(where, monkeypatch):
    monkeypatch.setenv("GKM_XFER_HYBRID", "1")  # the device census of raw chunks must catch it too
    rng = np.random.default_rng(where)
    sba, seg = genome(rng, 40 * B)
    sba[where] = ord("x")
    t = pinned_copy(sba)
    with pytest.raises(_native.GkError) as ei:
        load(t.numpy(), seg, monkeypatch, True, 1, 2)
    assert ei.value.code == _native.GK_E_ALPHABET


def test_set_sequence_waits_for_an_earlier_sort(monkeypatch):
    # a new sequence must not overwrite the resident one under a sort still queued on the stream
    rng = np.random.default_rng(3)
    a, seg = genome(rng, 30 * B)
    b, _ = genome(rng, 30 * B)
    eng = load(a, seg, monkeypatch, True)
    n = eng.enumerate(21)
    eng.sort(21)
    monkeypatch.setenv("GKM_PACK_MIN", "0")
    eng.set_sequence(b, seg)
    monkeypatch.delenv("GKM_PACK_MIN")
    np.testing.assert_array_equal(eng.copy_sequence(len(b)), b)
    n = eng.enumerate(21)
    eng.sort(21)
    want = oracle.quicksort(b, oracle.enumerate_starts(b, seg, 21), 21, 21, break_ties=True)
    np.testing.assert_array_equal(eng.copy_starts(np.empty(n, dtype=np.uint32)), want)


def test_packed_short_then_longer_sequence(monkeypatch):
    # a longer packed sequence after a shorter one grows the staging slots: the slots the earlier
    # transfer's unpacks read are freed only after the context's stream has drained (round-4 advice)
    rng = np.random.default_rng(23)
    a, seg = genome(rng, 3 * B + 5)
    b, segb = genome(rng, 70 * B + 11, contigs=3)
    monkeypatch.setenv("GKM_PACK_MIN", "0")
    monkeypatch.setenv("GKM_PACK_BLOCKS", "1")
    monkeypatch.setenv("GKM_XFER_THREADS", "2")
    eng = _native.Engine()
    eng.set_sequence(a, seg)
    monkeypatch.setenv("GKM_PACK_BLOCKS", "8")
    monkeypatch.setenv("GKM_XFER_THREADS", "6")
    eng.set_sequence(b, segb)
    for v in ("GKM_PACK_MIN", "GKM_PACK_BLOCKS", "GKM_XFER_THREADS"):
        monkeypatch.delenv(v)
    np.testing.assert_array_equal(eng.copy_sequence(len(b)), b)
    n = eng.enumerate(17)
    eng.sort(17)
    want = oracle.quicksort(b, oracle.enumerate_starts(b, segb, 17), 17, 17, break_ties=True)
    np.testing.assert_array_equal(eng.copy_starts(np.empty(n, dtype=np.uint32)), want)


@pytest.mark.parametrize("impl", ["scalar", "avx2", "avx512"])
def test_packer_implementations_agree(impl, monkeypatch):
    # the host packer's vector paths (GKM_PACK_IMPL; read once per process, so each run is a child)
    import subprocess
    import sys

    code = (
        "import numpy as np, sys; sys.path.insert(0, 'genome-kmers_amd'); from genome_kmers import _native\n"
        "rng = np.random.default_rng(5)\n"
        "s = np.frombuffer(b'ACGT', dtype=np.uint8)[rng.integers(0, 4, 3 * 65536 + 4321)].copy()\n"
        "s[70000:70010] = ord('N'); s[200000] = ord('$')\n"
        "seg = np.array([0, 200001], dtype=np.uint32)\n"
        "e = _native.Engine(); e.set_sequence(s, seg)\n"
        "assert np.array_equal(e.copy_sequence(len(s)), s) and not e.is_acgt()\n"
        "print('ok')\n")
    env = dict(__import__("os").environ, GKM_PACK_IMPL=impl, GKM_PACK_MIN="0", GKM_PACK_BLOCKS="1")
    from pathlib import Path
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=str(Path(__file__).resolve().parent.parent),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


# Round 5: the packed transfer leaves a 2-bit packed copy beside the resident sba (packed blocks'
# codes reordered, raw blocks packed from their bytes, the partial last word and the '$' pad packed
# after the transfer); msd_sort's L0 passes read it on an ACGT sba.  The sorted starts must equal
# the oracle's and the same sort without the copy (GKM_NO_RESIDENT_PACK=1), whatever the lengths,
# contig separators (raw blocks) and block / chunk boundaries.
@pytest.mark.parametrize("L,contigs", [(3 * B + 999, 3), (5 * B + 17, 1), (9 * B, 4), (B + 33, 2), (700_001, 1)])
@pytest.mark.parametrize("k,canonical", [(5, False), (21, False), (31, False), (32, True), (45, False), (45, True)])
def test_resident_packed_copy_sorts_like_the_oracle(L, contigs, k, canonical, monkeypatch):
    rng = np.random.default_rng(L + k)
    sba, seg = genome(rng, L, contigs=contigs)
    if L > 50_400 and not (sba[50_000:50_400] == ord("$")).any() and not (sba[1000:1400] == ord("$")).any():
        sba[1000:1400] = sba[50_000:50_400]  # a repeat: ties
    outs = []
    for res in (True, False):
        if not res:
            monkeypatch.setenv("GKM_NO_RESIDENT_PACK", "1")
        eng = load(sba, seg, monkeypatch, True, blocks=1, threads=2)
        assert eng.is_acgt()
        n = eng.enumerate(k)
        eng.sort(k, canonical=canonical)
        outs.append(eng.copy_starts(np.empty(n, dtype=np.uint32)))
        monkeypatch.delenv("GKM_NO_RESIDENT_PACK", raising=False)
    starts = oracle.enumerate_starts(sba, seg, k)
    want = oracle.canonical_sort(sba, starts, k) if canonical else oracle.quicksort(sba, starts, k, k, break_ties=True)
    np.testing.assert_array_equal(outs[0], want)
    np.testing.assert_array_equal(outs[1], want)
