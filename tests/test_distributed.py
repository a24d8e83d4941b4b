"""Multi-GPU path (genome_kmers.distributed): host logic, a world_size-2 gloo run on CPU, and the
device shard entry points with the exchange done in one process on one GPU.

The CPU run drives the real orchestration (histogram all_gather, bucket split, the exchange with
uneven splits in chunked point-to-point messages, receive pieces) with ``NumpyShardEngine``, a
test double that restates the engine's shard contract with numpy; the result is checked against
the oracle's break_ties=True order (oracle/, kmers.py:1654-1731).  The GPU test runs libgkm's gk_shard_partition /
gk_shard_sort for two ranks and checks the concatenation against gk_sort on the whole input.
"""

import os
import socket

import numpy as np
import pytest

from genome_kmers import distributed as D
from oracle import oracle
from genome_kmers import _native  # noqa: E402 (gk_set_option overrides)

K = 11


def _random_sba(L, seed, contigs=1):
    rng = np.random.default_rng(seed)
    parts = [np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, L // contigs)] for _ in range(contigs)]
    sba = parts[0]
    starts = [0]
    for p in parts[1:]:
        starts.append(len(sba) + 1)
        sba = np.concatenate([sba, np.frombuffer(b"$", dtype=np.uint8), p])
    return np.ascontiguousarray(sba), np.asarray(starts, dtype=np.uint32)


def _keys(sba, starts, k):
    code = np.zeros(256, dtype=np.uint64)
    for i, ch in enumerate(b"ACGT"):
        code[ch] = i
    key = np.zeros(len(starts), dtype=np.uint64)
    for j in range(k):
        key = (key << np.uint64(2)) | code[sba[starts + j]]
    return key


def _valid_starts(sba, seg, k, lo, hi):
    s = np.arange(lo, min(hi, len(sba)), dtype=np.int64)
    ok = np.ones(len(s), dtype=bool)
    for j in range(k):
        p = s + j
        inside = p < len(sba)
        ok &= inside
        ok[inside] &= sba[p[inside]] != 36
    return s[ok]


class NumpyShardEngine:
    """Test double of the engine's shard contract (include/gkm.h gk_shard_*), numpy on the host."""

    bits = 8

    def set_sequence(self, sba, seg):
        self.sba, self.seg = np.asarray(sba), np.asarray(seg)

    def sync(self):
        pass

    def shard_bucket_bits(self):
        return self.bits

    def shard_partition(self, lo, hi, k, keys_t, starts_t, canonical=False, starts_only=False):
        assert not canonical
        assert (keys_t is None) == starts_only, "a starts-only send has no key buffer"
        s = _valid_starts(self.sba, self.seg, k, lo, hi)
        key = _keys(self.sba, s, k)
        top = (key >> np.uint64(2 * k - self.bits)).astype(np.int64)
        order = np.argsort(top, kind="stable")
        n = len(s)
        if not starts_only:
            keys_t[:n] = __import__("torch").from_numpy(key[order].view(np.int64))
        starts_t[:n] = __import__("torch").from_numpy(s[order].astype(np.int32))
        return np.bincount(top, minlength=1 << self.bits).astype(np.uint64), n

    def shard_sort(self, keys_t, starts_t, n, k, off, ln, bk, canonical=False, starts_only=False):
        assert np.all(np.diff(bk.astype(np.int64)) >= 0), "pieces must come in bucket order"
        assert (keys_t is None) == starts_only, "a starts-only receive has no key buffer"
        st = starts_t[:n].numpy().astype(np.int64)
        # (starts only: the keys re-derived from the resident sequence, as the engine does)
        key = _keys(self.sba, st, k) if starts_only else keys_t[:n].numpy().view(np.uint64)
        idx = np.concatenate([np.arange(o, o + m) for o, m in zip(off.astype(np.int64), ln.astype(np.int64))]) \
            if len(off) else np.zeros(0, dtype=np.int64)
        key, st = key[idx], st[idx]
        order = np.argsort(key, kind="stable")  # the device sort is stable in piece order
        self.keys, self.starts = key[order], st[order]

    # key-range contract (gk_shard_histogram / gk_shard_sort_range): 12-bit top digits of 2-bit keys
    range_bits = 12

    def _top(self, key, k):
        return (key >> np.uint64(max(0, 2 * k - self.range_bits))).astype(np.int64)

    def shard_histogram(self, lo, hi, k, canonical=False):
        assert not canonical
        s = _valid_starts(self.sba, self.seg, k, lo, hi)
        return np.bincount(self._top(_keys(self.sba, s, k), k), minlength=1 << self.range_bits).astype(np.uint64), \
            self.range_bits

    def shard_sort_range(self, k, dlo, dhi, canonical=False):
        assert not canonical
        s = _valid_starts(self.sba, self.seg, k, 0, len(self.sba))
        key = _keys(self.sba, s, k)
        top = self._top(key, k)
        keep = (top >= dlo) & (top < dhi)
        key, s = key[keep], s[keep]
        order = np.argsort(key, kind="stable")  # the device sort is stable in start order
        self.keys, self.starts = key[order], s[order]
        return len(s)

    def is_acgt(self):
        return bool(np.isin(self.sba, np.frombuffer(b"ACGT$", dtype=np.uint8)).all())

    def materialize_keys(self):
        return 1  # the double keeps its sorted keys on the host

    def unique_count_only(self):
        return int(len(np.unique(self.keys)))


# ---- host logic --------------------------------------------------------------------------------
def test_count_kmers_matches_enumeration():
    sba, seg = _random_sba(3000, 1, contigs=3)
    assert D.count_kmers(len(sba), seg, K) == len(_valid_starts(sba, seg, K, 0, len(sba)))


def test_position_ranges_cover_and_align():
    for L, w in [(10_000, 2), (10_001, 3), (5, 4), (3_100_000_000, 8)]:
        b = D.position_ranges(L, w)
        assert b[0] == 0 and b[-1] == L and len(b) == w + 1
        assert all(x % 32 == 0 for x in b[:-1])
        assert all(b[i] <= b[i + 1] for i in range(w))


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_split_buckets_balanced_and_contiguous(world):
    rng = np.random.default_rng(world)
    totals = rng.integers(0, 1000, 256)
    b = D.split_buckets(totals, world)
    assert b[0] == 0 and b[-1] == 256 and all(b[i] <= b[i + 1] for i in range(world))
    share = [totals[b[r]:b[r + 1]].sum() for r in range(world)]
    assert sum(share) == totals.sum()
    assert max(share) <= totals.sum() / world + totals.max() + 1


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_split_buckets_min_max(world):
    # one heavy bucket (an assembly's N-run digit) between light ones: the largest range is the
    # smallest any contiguous split reaches (brute force over all boundaries at this size)
    import itertools

    rng = np.random.default_rng(10 + world)
    totals = rng.integers(0, 100, 14)
    totals[int(rng.integers(0, 14))] = 600
    b = D.split_buckets(totals, world)
    P = np.concatenate(([0], np.cumsum(totals)))
    got = max(P[b[r + 1]] - P[b[r]] for r in range(world))
    best = min(max(P[c[r + 1]] - P[c[r]] for r in range(world))
               for mid in itertools.combinations_with_replacement(range(15), world - 1)
               for c in [(0,) + mid + (14,)])
    assert got == best
    assert b[0] == 0 and b[-1] == 14 and all(b[i] <= b[i + 1] for i in range(world))


def test_split_buckets_skewed():
    totals = np.zeros(256, dtype=np.int64)
    totals[7] = 10_000
    b = D.split_buckets(totals, 4)
    assert b[0] == 0 and b[-1] == 256 and sum(totals[b[r]:b[r + 1]].sum() for r in range(4)) == 10_000


def test_receive_pieces_layout():
    H = np.array([[1, 2, 0, 3], [4, 0, 5, 6]])
    # rank owning buckets [1, 4): source 0 sends 2+0+3, source 1 sends 0+5+6
    off, ln, bk = D.receive_pieces(H, 1, 4, [5, 11])
    assert list(bk) == [1, 2, 3, 3]
    assert list(ln) == [2, 5, 3, 6]
    assert list(off) == [0, 5, 2, 10]


# ---- world_size 2 over gloo on CPU -------------------------------------------------------------
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, sba, seg, k, q, chunk, scheme="a2a", starts_only=None):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if scheme == "range":
            job = D.KeyRangeKmerSort(sba, seg, k, rank, world, engine=NumpyShardEngine(),
                                     torch_device=torch.device("cpu"))
        else:
            job = D.ShardedKmerSort(sba, seg, k, rank, world, engine=NumpyShardEngine(),
                                    torch_device=torch.device("cpu"), chunk=chunk, starts_only=starts_only)
        n_unique = job.run()
        q.put((rank, job.engine.starts.tolist(), n_unique, job.total_kmers, job.local_kmers))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("scheme,contigs,chunk,starts_only", [
    ("a2a", 1, None, None), ("a2a", 3, None, None), ("a2a", 1, 5000, None), ("a2a", 3, 5000, False),
    ("a2a", 1, None, False), ("range", 1, None, None), ("range", 3, None, None)])
def test_gloo_world2_matches_oracle(scheme, contigs, chunk, starts_only):
    import torch.multiprocessing as mp

    from oracle import oracle

    sba, seg = _random_sba(6000, 7 + contigs, contigs)
    # planted repeats: equal k-mers on both ranks (tie order across ranks)
    sba[4100:4200] = sba[100:200]  # (inside a contig: the '$' separators stay)
    sba[5000:5030] = sba[100:130]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, sba, seg, K, q, chunk, scheme, starts_only))
             for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = np.concatenate([np.asarray(r[1], dtype=np.uint32) for r in res])
    starts = oracle.enumerate_starts(sba, seg, K)
    want = oracle.quicksort(sba, starts, K, K, break_ties=True)
    assert res[0][3] == len(starts)
    assert sum(r[4] for r in res) == len(starts)
    np.testing.assert_array_equal(got, want)
    assert sum(r[2] for r in res) == len(np.unique(_keys(sba, starts.astype(np.int64), K)))


class ClassBGatherEngine(NumpyShardEngine):
    """A mixed-alphabet double for the class-B exchange of KeyRangeKmerSort: each rank reports
    made-up class-B lists of uneven sizes (one rank none) and the lists it is handed back are
    recorded; the sort itself is the ACGT double's."""

    def is_acgt(self):
        return False

    def shard_class_b(self, lo, hi, k, hist, canonical=False):
        r = int(lo // 1024)
        rest = np.arange(lo, lo + 3 * r, 3, dtype=np.uint32)
        runs = np.array([[lo + 1000 + j, 40 + j, ord("N")] for j in range(r % 3)], dtype=np.uint32).reshape(-1, 3)
        hist[0] += np.uint64(len(rest) + runs[:, 1].sum() // 2)
        return rest, runs

    def shard_sort_range_b(self, k, dlo, dhi, rest, runs, canonical=False):
        self.given = (rest.tolist(), runs.tolist())
        return self.shard_sort_range(k, dlo, dhi, canonical)


def _gather_worker(rank, world, port, sba, seg, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        job = D.KeyRangeKmerSort(sba, seg, K, rank, world, engine=ClassBGatherEngine(),
                                 torch_device=torch.device("cpu"))
        job.lo, job.hi = 1024 * rank, 1024 * (rank + 1)  # (the double derives its lists from lo)
        job.run()
        q.put((rank, job.engine.given))
    finally:
        dist.destroy_process_group()


def test_gloo_class_b_lists_gathered_in_rank_order():
    """KeyRangeKmerSort on a mixed sba: every rank receives the concatenation, in rank order, of
    every rank's class-B lists (uneven sizes, an empty rank, runs as triples) over gloo."""
    import torch.multiprocessing as mp

    sba, seg = _random_sba(6000, 5)
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, sba, seg, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_rest, want_runs = [], []
    for r in range(world):
        want_rest += list(range(1024 * r, 1024 * r + 3 * r, 3))
        want_runs += [[1024 * r + 1000 + j, 40 + j, ord("N")] for j in range(r % 3)]
    for _, (rest, runs) in res:
        assert rest == want_rest and runs == want_runs


# ---- device shard entry points, two ranks in one process ---------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("world,contigs,k,canonical,iupac", [
    (2, 1, 31, False, False), (3, 4, 31, False, False), (2, 3, 63, False, False), (3, 2, 31, True, False),
    (2, 2, 63, True, True), (2, 1, 40, False, True)])
def test_gpu_shards_concatenate_to_single_sort(world, contigs, k, canonical, iupac):
    import torch

    from genome_kmers import _native

    sba, seg = _random_sba(200_000 + 17, 3 + world, contigs)
    sba[150_100:151_000] = sba[1000:1900]  # repeats across ranks (inside a contig)
    sba[160_000:160_900] = oracle.reverse_complement(sba[1000:1900])  # reverse-complement repeat
    if iupac:
        sba[5000:5100] = ord("N")
        sba[90_000:90_050:7] = ord("R")
    engines = [_native.Engine(0) for _ in range(world)]
    bounds = D.position_ranges(len(sba), world)
    dev = torch.device("cuda", 0)
    sends, hists = [], []
    for r, e in enumerate(engines):
        e.set_sequence(sba, seg)
        cap = bounds[r + 1] - bounds[r] + 64
        sk = torch.empty(cap, dtype=torch.int64, device=dev)
        sv = torch.empty(cap, dtype=torch.int32, device=dev)
        hist, n = e.shard_partition(bounds[r], bounds[r + 1], k, sk, sv, canonical=canonical)
        sends.append((sk, sv, n))
        hists.append(np.asarray(hist, dtype=np.int64))
    H = np.stack(hists)
    bb = D.split_buckets(H.sum(axis=0), world)
    got, uniq = [], 0
    for r, e in enumerate(engines):
        parts_k, parts_v, recv_counts = [], [], []
        for s in range(world):
            lo = int(H[s, :bb[r]].sum())
            m = int(H[s, bb[r]:bb[r + 1]].sum())
            parts_k.append(sends[s][0][lo:lo + m])
            parts_v.append(sends[s][1][lo:lo + m])
            recv_counts.append(m)
        R = sum(recv_counts)
        rk = torch.cat(parts_k + [torch.empty(64, dtype=torch.int64, device=dev)])
        rv = torch.cat(parts_v + [torch.empty(64, dtype=torch.int32, device=dev)])
        off, ln, bk = D.receive_pieces(H, bb[r], bb[r + 1], recv_counts)
        torch.cuda.current_stream(dev).synchronize()
        e.shard_sort(rk, rv, R, k, off, ln, bk, canonical=canonical)
        got.append(e.copy_starts())
        uniq += e.unique_count_only()
    ref = _native.Engine(0)
    ref.set_sequence(sba, seg)
    ref.enumerate(k)
    ref.sort(k, canonical=canonical)
    np.testing.assert_array_equal(np.concatenate(got), ref.copy_starts())
    assert uniq == ref.unique_count_only()


# Round 6: starts-only shards (GK_SHARD_STARTS_ONLY): the send holds no keys, the receiver re-derives
# them from its own copy of the sequence -- with and without the transfer's resident packed copy
@pytest.mark.gpu
@pytest.mark.parametrize("packed", [False, True], ids=["packed_now", "resident"])
@pytest.mark.parametrize("world,contigs,k", [(2, 1, 31), (3, 4, 31), (8, 1, 31), (4, 2, 12), (5, 3, 32), (2, 1, 5)])
def test_gpu_shards_starts_only(world, contigs, k, packed, monkeypatch):
    import torch

    from genome_kmers import _native

    if packed:
        monkeypatch.setenv("GKM_PACK_MIN", "0")
        monkeypatch.setenv("GKM_PACK_BLOCKS", "1")
    sba, seg = _random_sba(200_000 + 17, 5 + world, contigs)
    sba[150_100:151_000] = sba[1000:1900]  # repeats across ranks (inside a contig)
    engines = [_native.Engine(0) for _ in range(world)]
    bounds = D.position_ranges(len(sba), world)
    dev = torch.device("cuda", 0)
    sends, hists = [], []
    for r, e in enumerate(engines):
        e.set_sequence(sba, seg)
        assert e.resident_packed() == packed
        sv = torch.empty(bounds[r + 1] - bounds[r] + 64, dtype=torch.int32, device=dev)
        hist, n = e.shard_partition(bounds[r], bounds[r + 1], k, None, sv, starts_only=True)
        sends.append(sv)
        hists.append(np.asarray(hist, dtype=np.int64))
    H = np.stack(hists)
    bb = D.split_buckets(H.sum(axis=0), world)
    got, keys, uniq = [], [], 0
    for r, e in enumerate(engines):
        parts_v, recv_counts = [], []
        for s in range(world):
            lo = int(H[s, :bb[r]].sum())
            m = int(H[s, bb[r]:bb[r + 1]].sum())
            parts_v.append(sends[s][lo:lo + m])
            recv_counts.append(m)
        R = sum(recv_counts)
        rv = torch.cat(parts_v + [torch.empty(64, dtype=torch.int32, device=dev)])
        off, ln, bk = D.receive_pieces(H, bb[r], bb[r + 1], recv_counts)
        torch.cuda.current_stream(dev).synchronize()
        e.shard_sort(None, rv, R, k, off, ln, bk, starts_only=True)
        got.append(e.copy_starts())
        keys.append(e.copy_keys())
        uniq += e.unique_count_only()
    ref = _native.Engine(0)
    ref.set_sequence(sba, seg)
    ref.enumerate(k)
    ref.sort(k)
    np.testing.assert_array_equal(np.concatenate(got), ref.copy_starts())
    np.testing.assert_array_equal(np.concatenate(keys), ref.copy_keys())
    assert uniq == ref.unique_count_only()


@pytest.mark.gpu
def test_gpu_shards_starts_only_refuses_what_it_cannot_rederive():
    import torch

    from genome_kmers import _native

    sba, seg = _random_sba(50_000, 3, 1)
    sv = torch.empty(60_000, dtype=torch.int32, device=torch.device("cuda", 0))
    e = _native.Engine(0)
    e.set_sequence(sba, seg)
    for k, canonical in [(33, False), (31, True)]:
        with pytest.raises(_native.GkError, match="starts-only"):
            e.shard_partition(0, len(sba), k, None, sv, canonical=canonical, starts_only=True)
    sba[100:110] = ord("N")
    e.set_sequence(sba, seg)
    with pytest.raises(_native.GkError, match="starts-only"):
        e.shard_partition(0, len(sba), 31, None, sv, starts_only=True)


@pytest.mark.gpu
@pytest.mark.parametrize("world,contigs,k,canonical,iupac", [
    (2, 1, 31, False, False), (3, 4, 31, False, False), (8, 1, 31, False, False), (2, 3, 63, False, False),
    (3, 2, 31, True, False), (2, 2, 63, True, True), (2, 1, 40, False, True), (4, 2, 21, False, False),
    (5, 3, 31, False, True), (8, 2, 31, True, True), (3, 1, 5, False, True)])
def test_gpu_key_ranges_concatenate_to_single_sort(world, contigs, k, canonical, iupac):
    """gk_shard_histogram / gk_shard_sort_range for every rank of a world in one process: the
    ranks' sorted starts, concatenated in rank order, equal gk_sort on the whole input."""
    from genome_kmers import _native

    sba, seg = _random_sba(200_000 + 17, 3 + world, contigs)
    sba[150_100:151_000] = sba[1000:1900]  # repeats in different position shares
    sba[160_000:160_900] = oracle.reverse_complement(sba[1000:1900])
    if iupac:
        sba[5000:5100] = ord("N")
        sba[90_000:90_050:7] = ord("R")
        sba[120_000:120_300] = ord("N")  # N runs longer than k: homopolymer groups
        sba[130_000:130_080] = ord("Y")
        sba[140_000:140_090] = ord("R")  # complement of Y: one canonical group with it
    bounds = D.position_ranges(len(sba), world)
    e = _native.Engine(0)
    e.set_sequence(sba, seg)
    hist = None
    for r in range(world):
        h, bits = e.shard_histogram(bounds[r], bounds[r + 1], k, canonical=canonical)
        hist = h.astype(np.int64) if hist is None else hist + h.astype(np.int64)
    assert bits == min(12, 2 * k)  # ownership digits: the top 12 bits of the (ACGT-only k-mers') 2-bit keys
    total = D.count_kmers(len(sba), seg, k)
    if iupac:  # the digits count the ACGT-only k-mers; the others follow their byte-order interval
        assert 0 < int(hist.sum()) < total
    else:
        assert int(hist.sum()) == total
    db = D.split_buckets(hist, world)
    got, keys, uniq, kept = [], [], 0, 0
    for r in range(world):
        kept += e.shard_sort_range(k, db[r], db[r + 1], canonical=canonical)
        got.append(e.copy_starts())
        keys.append(e.copy_keys())
        uniq += e.unique_count_only()
    assert kept == total
    ref = _native.Engine(0)
    ref.set_sequence(sba, seg)
    ref.enumerate(k)
    ref.sort(k, canonical=canonical)
    np.testing.assert_array_equal(np.concatenate(got), ref.copy_starts())
    np.testing.assert_array_equal(np.concatenate(keys), ref.copy_keys())
    assert uniq == ref.unique_count_only()


# Round 5: the ranks' levels write packed pairs where the bits fit (msd_sort_range, msd_shard_sort);
# at test sizes GKM_TEST_PAIRS=1 makes every level that can write them do so
@pytest.mark.gpu
@pytest.mark.parametrize("world,contigs,k,canonical,iupac", [
    (2, 1, 31, False, False), (3, 2, 31, True, False), (2, 2, 63, True, True), (8, 2, 31, True, True)])
def test_gpu_key_ranges_packed_pairs(world, contigs, k, canonical, iupac, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_TEST_PAIRS", "1")
    test_gpu_key_ranges_concatenate_to_single_sort(world, contigs, k, canonical, iupac)


# Round 5: a rank keeping at least half of the ownership digits (<= 2 ranks by default) fuses its select into the L0
# (msd0_pipe_kernel<..., OWN>); GKM_RANGE_FUSED=0/1 forces either path at any world size
@pytest.mark.gpu
@pytest.mark.parametrize("fused", ["0", "1"], ids=["select", "fused"])
@pytest.mark.parametrize("world,contigs,k,canonical,iupac", [
    (2, 1, 31, False, False), (8, 1, 31, False, False), (3, 2, 31, True, False), (2, 2, 63, True, True),
    (5, 3, 31, False, True), (3, 1, 5, False, True), (4, 2, 21, False, False)])
def test_gpu_key_ranges_fused_select(fused, world, contigs, k, canonical, iupac, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_RANGE_FUSED", fused)
    test_gpu_key_ranges_concatenate_to_single_sort(world, contigs, k, canonical, iupac)


# Round 5: through the packed transfer (GKM_PACK_MIN=0) the ranks' select, histogram and fused L0
# read the resident 2-bit packed copy of the sequence (stops = non-ACGT bytes: class A of a mixed sba);
# round 6: forward keys of <= 32 symbols take the SWAR select over it (msd0_rsel_kernel)
@pytest.mark.gpu
@pytest.mark.parametrize("world,contigs,k,canonical,iupac", [
    (2, 1, 31, False, False), (5, 3, 31, False, True), (8, 2, 31, True, True), (2, 2, 63, True, True),
    (3, 1, 21, False, False), (8, 1, 31, False, False), (3, 1, 5, False, True), (4, 2, 32, False, False),
    (7, 2, 16, False, True), (6, 3, 3, False, False)])
def test_gpu_key_ranges_resident_packed_copy(world, contigs, k, canonical, iupac, monkeypatch):
    monkeypatch.setenv("GKM_PACK_MIN", "0")
    monkeypatch.setenv("GKM_PACK_BLOCKS", "1")
    test_gpu_key_ranges_concatenate_to_single_sort(world, contigs, k, canonical, iupac)


# Round 6: the ownership-digit histogram over the packed copy (own_hist_rsel_kernel) against numpy,
# shares whose bounds are not multiples of 32, stops from contig ends and non-ACGT runs
@pytest.mark.gpu
@pytest.mark.parametrize("k", [3, 5, 16, 31, 32])
@pytest.mark.parametrize("iupac", [False, True])
def test_gpu_shard_histogram_packed_copy_vs_numpy(k, iupac, monkeypatch):
    from genome_kmers import _native

    if iupac and k < 4:
        pytest.skip("a mixed sba with k < 4 takes 4-bit keys (no split, not the packed path)")
    monkeypatch.setenv("GKM_PACK_MIN", "0")
    monkeypatch.setenv("GKM_PACK_BLOCKS", "1")
    sba, seg = _random_sba(150_000 + 13, 41 + k, 3)
    if iupac:
        sba[7000:7100] = ord("N")
        sba[60_000:60_040:3] = ord("R")
    e = _native.Engine(0)
    e.set_sequence(sba, seg)
    ob = min(12, 2 * k)
    code = np.full(256, 255, dtype=np.int64)
    for i, ch in enumerate(b"ACGT"):
        code[ch] = i
    c = code[sba]
    L = len(sba)
    for lo, hi in [(0, L), (32, 70_001), (64, 64 + 32 * 7 + 5), (99_968, L), (4096, 4097)]:  # (lo: multiples of 32)
        h, bits = e.shard_histogram(lo, hi, k, canonical=False)
        assert bits == ob
        p = np.arange(lo, min(hi, L - k + 1))
        ok = np.ones(len(p), dtype=bool)
        dig = np.zeros(len(p), dtype=np.int64)
        for j in range(k):
            cj = c[p + j]
            ok &= cj != 255
            if 2 * j < ob:
                dig = (dig << 2) | np.where(cj == 255, 0, cj)
        want = np.bincount(dig[ok], minlength=1 << ob)
        np.testing.assert_array_equal(np.asarray(h, dtype=np.int64)[:1 << ob], want)


# Round 6: the compacting rank L0 (own_count_kernel / own_part_kernel: test, compact, then rank the
# kept k-mers only), opt-in (GKM_OWN_L0_COMPACT=1), at fused and select-sized shares
@pytest.mark.gpu
@pytest.mark.parametrize("world,contigs,k,iupac", [(2, 1, 31, False), (8, 2, 31, False), (5, 3, 31, True),
                                                   (3, 1, 12, False), (4, 2, 32, True), (16, 1, 31, False)])
def test_gpu_key_ranges_compacting_l0(world, contigs, k, iupac, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_OWN_L0_COMPACT", "1")
    monkeypatch.setitem(_native.options, "GKM_RANGE_FUSED", "1")
    monkeypatch.setenv("GKM_PACK_MIN", "0")
    monkeypatch.setenv("GKM_PACK_BLOCKS", "1")
    test_gpu_key_ranges_concatenate_to_single_sort(world, contigs, k, False, iupac)


@pytest.mark.gpu
@pytest.mark.parametrize("world,k,canonical", [(2, 31, False), (2, 63, True)])
def test_gpu_key_ranges_fused_packed_l0(world, k, canonical, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_RANGE_FUSED", "1")
    monkeypatch.setitem(_native.options, "GKM_TEST_P88", "1")
    monkeypatch.setitem(_native.options, "GKM_TEST_PAIRS", "1")
    test_gpu_key_ranges_concatenate_to_single_sort(world, 1, k, canonical, False)


@pytest.mark.gpu
@pytest.mark.parametrize("world,contigs,k,canonical,iupac", [(2, 1, 31, False, False), (3, 2, 31, True, False),
                                                             (2, 2, 63, True, True)])
def test_gpu_shards_packed_pairs(world, contigs, k, canonical, iupac, monkeypatch):
    monkeypatch.setitem(_native.options, "GKM_TEST_PAIRS", "1")
    test_gpu_shards_concatenate_to_single_sort(world, contigs, k, canonical, iupac)


@pytest.mark.gpu
@pytest.mark.parametrize("world,contigs,k,canonical", [
    (2, 2, 63, True), (2, 1, 40, False), (5, 3, 31, False), (8, 2, 31, True), (3, 1, 5, False), (4, 2, 6, False)])
def test_gpu_key_ranges_class_b_given(world, contigs, k, canonical):
    """gk_shard_class_b per position share + gk_shard_sort_range_b with the gathered lists (no
    whole-sequence class-B scan per rank): the histogram gains every class-B k-mer (homopolymers at
    11/16 weight), the ranks keep every k-mer exactly once, and their concatenation is gk_sort's."""
    from genome_kmers import _native

    sba, seg = _random_sba(200_000 + 17, 3 + world, contigs)
    sba[150_100:151_000] = sba[1000:1900]
    sba[160_000:160_900] = oracle.reverse_complement(sba[1000:1900])
    sba[5000:5100] = ord("N")
    sba[90_000:90_050:7] = ord("R")
    sba[120_000:120_300] = ord("N")
    sba[130_000:130_080] = ord("Y")
    sba[140_000:140_090] = ord("R")
    bounds = D.position_ranges(len(sba), world)
    bounds[1] = 120_128 if world == 2 else bounds[1]  # a homopolymer run across a share boundary
    e = _native.Engine(0)
    e.set_sequence(sba, seg)
    hist, rests, runs_l, plain = None, [], [], None
    for r in range(world):
        h, bits = e.shard_histogram(bounds[r], bounds[r + 1], k, canonical=canonical)
        h = np.asarray(h, dtype=np.uint64)
        h0 = h.astype(np.int64)
        plain = h0 if plain is None else plain + h0
        rest, runs = e.shard_class_b(bounds[r], bounds[r + 1], k, h, canonical=canonical)
        assert np.all(rest >= bounds[r]) and np.all(rest < bounds[r + 1])
        assert np.all(np.diff(rest.astype(np.int64)) > 0)
        if len(runs):
            assert np.all(runs[:, 0] >= bounds[r]) and np.all(runs[:, 0] < bounds[r + 1])
        added = int(h.astype(np.int64).sum()) - int(h0.sum())
        assert added == len(rest) + sum((int(c) * 11 + 15) // 16 for c in runs[:, 1])
        hist = h.astype(np.int64) if hist is None else hist + h.astype(np.int64)
        rests.append(rest)
        runs_l.append(runs)
    rest_all, runs_all = np.concatenate(rests), np.concatenate(runs_l).reshape(-1, 3)
    total = D.count_kmers(len(sba), seg, k)
    # every non-ACGT k-mer is in exactly one list entry
    assert int(plain.sum()) + len(rest_all) + int(runs_all[:, 1].sum()) == total
    db = D.split_buckets(hist, world)
    got, keys, uniq, kept = [], [], 0, 0
    for r in range(world):
        kept += e.shard_sort_range_b(k, db[r], db[r + 1], rest_all, runs_all, canonical=canonical)
        got.append(e.copy_starts())
        keys.append(e.copy_keys())
        uniq += e.unique_count_only()
    assert kept == total
    ref = _native.Engine(0)
    ref.set_sequence(sba, seg)
    ref.enumerate(k)
    ref.sort(k, canonical=canonical)
    np.testing.assert_array_equal(np.concatenate(got), ref.copy_starts())
    np.testing.assert_array_equal(np.concatenate(keys), ref.copy_keys())
    assert uniq == ref.unique_count_only()


@pytest.mark.gpu
@pytest.mark.parametrize("world,k,canonical", [(4, 31, False), (7, 25, False), (4, 31, True), (3, 63, True)])
def test_gpu_key_range_repeated_calls(world, k, canonical):
    """Repeated gk_shard_sort_range calls on one engine over hundreds of select tiles, ranges in
    growing then shrinking size order (buffers grown, then reused): each call keeps exactly its
    histogram's k-mers, repeats its own first result, and the ranks concatenate to gk_sort."""
    from genome_kmers import _native

    sba, seg = _random_sba(3_000_017, 11 + world, 1)
    sba[2_000_000:2_004_000] = sba[10_000:14_000]  # ties across distant tiles
    bounds = D.position_ranges(len(sba), world)
    e = _native.Engine(0)
    e.set_sequence(sba, seg)
    hist = None
    for r in range(world):
        h, _ = e.shard_histogram(bounds[r], bounds[r + 1], k, canonical=canonical)
        hist = h.astype(np.int64) if hist is None else hist + h.astype(np.int64)
    db = D.split_buckets(hist, world)
    order = sorted(range(world), key=lambda r: int(hist[db[r]:db[r + 1]].sum()))  # growing ranges
    got = {}
    for r in order + order[::-1]:
        n = e.shard_sort_range(k, db[r], db[r + 1], canonical=canonical)
        assert n == int(hist[db[r]:db[r + 1]].sum())
        starts = e.copy_starts()
        if r in got:
            np.testing.assert_array_equal(starts, got[r])
        got[r] = starts
    ref = _native.Engine(0)
    ref.set_sequence(sba, seg)
    ref.enumerate(k)
    ref.sort(k, canonical=canonical)
    np.testing.assert_array_equal(np.concatenate([got[r] for r in range(world)]), ref.copy_starts())


def _gpu_a2a_worker(rank, world, port, sba, seg, k, canonical, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # device send / receive buffers, the exchange staged through host memory (gloo)
        job = D.ShardedKmerSort(sba, seg, k, rank, world, device=0, torch_device=torch.device("cuda", 0),
                                canonical=canonical, chunk=1 << 16)
        assert job.stage_host
        u = job.run()
        q.put((rank, job.engine.copy_starts().tolist(), u, job.local_kmers))
    except Exception as exc:  # report instead of leaving the parent waiting
        q.put((rank, repr(exc), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("k,canonical,iupac", [(31, False, False), (63, False, True), (31, True, False)])
def test_gpu_all_to_all_two_processes(k, canonical, iupac):
    """The north star's exchange path as two real processes, each with its own libgkm engine on GPU
    0: gk_shard_partition of the rank's position share, the all-to-all of (key, start) over gloo
    (device buffers staged through the host, messages of 64 KiB), gk_shard_sort of the received
    buckets; the rank-ordered concatenation equals the single-GPU sort."""
    import torch.multiprocessing as mp

    from genome_kmers import _native

    sba, seg = _random_sba(300_000 + 5, 13, 3)
    sba[250_000:251_000] = sba[2000:3000]  # a repeat across ranks (inside the third contig)
    sba[150_000:150_900] = oracle.reverse_complement(sba[5000:5900])
    if iupac:
        sba[60_000:60_400] = ord("N")
        sba[90_000:90_050:7] = ord("R")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_a2a_worker, args=(r, 2, port, sba, seg, k, canonical, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(r[2] is not None for r in res), res
    assert all(p.exitcode == 0 for p in procs)
    ref = _native.Engine(0)
    ref.set_sequence(sba, seg)
    n = ref.enumerate(k)
    ref.sort(k, canonical=canonical)
    assert sum(r[3] for r in res) == n
    np.testing.assert_array_equal(np.concatenate([np.asarray(r[1], dtype=np.uint32) for r in res]), ref.copy_starts())
    assert sum(r[2] for r in res) == ref.unique_count_only()


def _gpu_range_worker(rank, world, port, sba, seg, k, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        job = D.KeyRangeKmerSort(sba, seg, k, rank, world, device=0, torch_device=torch.device("cpu"))
        u = job.run()
        q.put((rank, job.engine.copy_starts().tolist(), u, job.local_kmers))
    except Exception as exc:  # report instead of leaving the parent waiting
        q.put((rank, repr(exc), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("iupac", [False, True])
def test_gpu_key_range_two_processes(iupac):
    """Two ranks as separate processes (gloo for the 2 KiB all-reduce), each with its own libgkm
    engine on GPU 0: the rank-ordered concatenation equals the single-GPU sort."""
    import torch.multiprocessing as mp

    from genome_kmers import _native

    sba, seg = _random_sba(300_000 + 5, 11, 3)
    sba[250_000:251_000] = sba[2000:3000]  # a repeat across contigs (inside the third one)
    if iupac:  # class-B lists gathered over gloo (gk_shard_class_b / gk_shard_sort_range_b)
        sba[60_000:60_400] = ord("N")
        sba[149_000:151_000] = ord("N")  # across the two position shares
        sba[90_000:90_050:7] = ord("R")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_range_worker, args=(r, 2, port, sba, seg, 31, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(r[2] is not None for r in res), res
    assert all(p.exitcode == 0 for p in procs)
    ref = _native.Engine(0)
    ref.set_sequence(sba, seg)
    ref.enumerate(31)
    ref.sort(31)
    np.testing.assert_array_equal(np.concatenate([np.asarray(r[1], dtype=np.uint32) for r in res]), ref.copy_starts())
    assert sum(r[2] for r in res) == ref.unique_count_only()
