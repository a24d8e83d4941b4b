"""Multi-GPU k-mer sort: one process per GPU under torch.distributed.

The reference sorts in one process (``Kmers.sort``, kmers.py:1624-1652); this module is one rank's
share of the same result on N GPUs.  Every rank holds the whole sequence byte array in HBM and owns
one contiguous range of top key digits, so the ranks' sorted starts, concatenated in rank order,
are ``Kmers.sort``'s order with ``break_ties=True`` (kmers.py:1710-1711) -- the single-GPU order --
and unique counts stay local (equal keys share a digit).  Two drivers:

``KeyRangeKmerSort`` (default): no k-mer moves between GPUs.  Histograms of the rank's position
share are all-reduced (4096 12-bit ownership digits, 32 KiB), the digits are cut into ranges of about n/N k-mers, and each rank
selects its k-mers from the whole resident sequence and sorts them.

``ShardedKmerSort`` (all-to-all):
1. ``shard_partition``: the rank encodes the k-mers that START in its position range
   [lo_r, lo_r+1) (cut at multiples of 32; a k-mer near hi reads a (k-1)-base halo) and
   partitions them stably by the top ``bits`` (8) key bits into a torch-owned send buffer;
2. ``all_gather`` of the 256-bucket histograms: every rank derives the same split of the buckets
   into N contiguous ranges of about n/N k-mers each (``split_buckets``);
3. the exchange: every rank sends each other rank the buckets it owns as one group of
   point-to-point messages (ncclSend / ncclRecv over xGMI under RCCL) -- keys and starts, or (round
   6, ``starts_only``: forward keys of an A/C/G/T sequence with k <= 32, the default there) the
   starts alone, 4 B per k-mer instead of 12: every rank holds the whole sequence, so the receiver
   re-derives each key from its own copy (GK_SHARD_STARTS_ONLY);
4. ``shard_sort``: the received buckets are sorted by the MSD levels below the top bits.  A bucket
   arrives as one piece per source rank; pieces are listed in source-rank order, and ranks own
   ascending positions, so equal keys stay in ascending start order.
"""

from __future__ import annotations

import time

import numpy as np


def count_kmers(sba_len: int, seg_starts: np.ndarray, k: int) -> int:
    """n = sum over contigs of max(0, len - k + 1) (kmers.py:837-861); contig s covers
    [starts[s], starts[s+1] - 2], the last one ends at sba_len - 1."""
    starts = np.asarray(seg_starts, dtype=np.int64)
    ends = np.append(starts[1:] - 2, sba_len - 1)
    return int(np.maximum(ends - starts + 1 - k + 1, 0).sum())


def position_ranges(sba_len: int, world: int) -> list[int]:
    """world + 1 boundaries of equal start-position ranges, cut at multiples of 32."""
    return [(sba_len * r // world) // 32 * 32 for r in range(world)] + [sba_len]


def split_buckets(totals: np.ndarray, world: int) -> list[int]:
    """world + 1 bucket boundaries: rank r receives buckets [b_r, b_r+1).  The largest range is as
    small as contiguous ranges allow (binary search on the capacity; a greedy fill decides whether
    a capacity fits), and each boundary is the one nearest an even share of what is left that keeps
    the rest within that capacity -- so one heavy bucket (the N runs' digit of an assembly) costs
    its own rank alone, where cutting at the prefixes r/world of the total gave that rank the whole
    bucket on top of its share."""
    t = np.asarray(totals, dtype=np.int64)
    nb = len(t)
    P = np.concatenate(([0], np.cumsum(t)))  # P[i]: the buckets before i
    n = int(P[-1])
    if world <= 1 or n == 0:
        return [0] * world + [nb]

    def last_fit(s, cap):  # the furthest boundary e with buckets [s, e) holding <= cap
        return int(np.searchsorted(P, P[s] + cap, side="right")) - 1

    def fits(s, ranks, cap):  # buckets [s, nb) in `ranks` ranges of <= cap
        for _ in range(ranks):
            if s >= nb:
                return True
            s = last_fit(s, cap)
        return s >= nb

    lo, hi = max(-(-n // world), int(t.max())), n
    while lo < hi:
        mid = (lo + hi) // 2
        if fits(0, world, mid):
            hi = mid
        else:
            lo = mid + 1
    cap = lo
    bounds, s = [0], 0
    for r in range(world - 1):
        left = world - r
        want = P[s] + (n - P[s]) / left
        e_max = last_fit(s, cap)
        near = int(np.searchsorted(P, want, side="left"))
        cands = sorted({min(near, e_max), min(max(near - 1, s), e_max)}, key=lambda e: abs(P[e] - want))
        e = next(e for e in cands + [e_max] if fits(e, left - 1, cap))
        bounds.append(e)
        s = e
    bounds.append(nb)
    return bounds


def receive_pieces(H: np.ndarray, b0: int, b1: int, recv_counts: list[int]):
    """Pieces (offset, length, bucket) of the receive buffer for buckets [b0, b1): source s's
    chunk starts at the exclusive prefix of recv_counts and holds its buckets in order."""
    world = H.shape[0]
    recv_off = np.concatenate(([0], np.cumsum(recv_counts)[:-1])).astype(np.int64)
    off, ln, bk = [], [], []
    within = np.zeros(world, dtype=np.int64)
    for b in range(b0, b1):
        for s in range(world):
            m = int(H[s, b])
            if m:
                off.append(int(recv_off[s] + within[s]))
                ln.append(m)
                bk.append(b)
            within[s] += m
    return (np.asarray(off, dtype=np.uint64), np.asarray(ln, dtype=np.uint64), np.asarray(bk, dtype=np.uint32))


class ShardedKmerSort:
    """One rank of the N-GPU sort of the fixed-length k-mers of a sequence (min = max = k).

    ``engine`` defaults to a ``genome_kmers._native.Engine`` on ``device`` (HIP, no fallback);
    ``torch_device`` is where the exchange buffers live (the GPU by default).
    """

    def __init__(self, sba: np.ndarray, seg_starts: np.ndarray, k: int, rank: int, world: int, device: int = 0,
                 engine=None, torch_device=None, group=None, chunk: int = None, canonical: bool = False,
                 stage_host: bool = None, starts_only: bool = None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.group = torch, dist, group
        self.rank, self.world, self.k = rank, world, k
        self.canonical = canonical  # canonical k-mers (Kmers.sort(canonical=True)); same flag on every rank
        self.dev = torch_device if torch_device is not None else torch.device("cuda", device)
        if engine is None:
            from genome_kmers import _native

            engine = _native.Engine(device)
        self.engine = engine
        t0 = time.perf_counter()
        self.engine.set_sequence(sba, seg_starts)
        self.engine.sync()
        self.h2d_ms = (time.perf_counter() - t0) * 1e3
        bounds = position_ranges(len(sba), world)
        self.lo, self.hi = bounds[rank], bounds[rank + 1]
        self.total_kmers = count_kmers(len(sba), seg_starts, k)
        self.nb = 1 << self.engine.shard_bucket_bits()
        # only the starts cross the exchange where the receiver can re-derive the keys (the same
        # decision on every rank: the same sequence, k and flag)
        if starts_only is None:
            starts_only = not canonical and k <= 32 and self.engine.is_acgt()
        self.starts_only = starts_only
        cap = self.hi - self.lo + 64
        self.send_k = None if starts_only else torch.empty(cap, dtype=torch.int64, device=self.dev)
        self.send_v = torch.empty(cap, dtype=torch.int32, device=self.dev)
        self.recv_k = torch.empty(0, dtype=torch.int64, device=self.dev)
        self.recv_v = torch.empty(0, dtype=torch.int32, device=self.dev)
        self.local_kmers = 0
        self.bucket_bounds = None
        if chunk:
            self.CHUNK_BYTES = chunk
        # device buffers over a backend without device point-to-point (gloo): the exchange is
        # staged through host copies of the send and receive segments
        if stage_host is None:
            stage_host = self.dev.type != "cpu" and dist.is_initialized() and dist.get_backend(group) == "gloo"
        self.stage_host = stage_host

    def _ensure_recv(self, n: int):
        if self.recv_v.numel() < n + 64:
            size = n + n // 8 + 64
            if not self.starts_only:
                self.recv_k = self.torch.empty(size, dtype=self.torch.int64, device=self.dev)
            self.recv_v = self.torch.empty(size, dtype=self.torch.int32, device=self.dev)

    # bytes per point-to-point message: RCCL mis-copies messages of 2^31 bytes and more (measured
    # with world-1 all_to_all_single: half the elements wrong at >= 2 GiB, tools/a2a_probe.py)
    CHUNK_BYTES = 1 << 30

    def _exchange(self, send, recv, send_counts, recv_counts):
        """The all-to-all of the per-destination segments of ``send`` into the per-source segments
        of ``recv``: one group of point-to-point sends / receives (ncclSend / ncclRecv over xGMI
        under RCCL), each message at most CHUNK_BYTES; the rank's own segment is a local copy."""
        dist = self.dist
        so = np.concatenate(([0], np.cumsum(send_counts)[:-1])).astype(np.int64)
        ro = np.concatenate(([0], np.cumsum(recv_counts)[:-1])).astype(np.int64)
        if self.stage_host:
            dev_recv = recv
            send = send[:int(np.sum(send_counts))].cpu()
            recv = self.torch.empty(int(np.sum(recv_counts)), dtype=recv.dtype)
        step = max(1, self.CHUNK_BYTES // send.element_size())
        me = self.rank
        ops = []
        for r in range(self.world):
            if r == me:
                continue
            for a in range(0, int(send_counts[r]), step):
                m = min(step, int(send_counts[r]) - a)
                ops.append(dist.P2POp(dist.isend, send[so[r] + a:so[r] + a + m], r, group=self.group))
            for a in range(0, int(recv_counts[r]), step):
                m = min(step, int(recv_counts[r]) - a)
                ops.append(dist.P2POp(dist.irecv, recv[ro[r] + a:ro[r] + a + m], r, group=self.group))
        m = int(send_counts[me])
        if m:
            recv[ro[me]:ro[me] + m].copy_(send[so[me]:so[me] + m])
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        if self.stage_host and recv.numel():
            dev_recv[:recv.numel()].copy_(recv)

    def run(self) -> int:
        """One sort; returns this rank's number of distinct k-mers."""
        torch, dist = self.torch, self.dist
        hist, n = self.engine.shard_partition(self.lo, self.hi, self.k, self.send_k, self.send_v,
                                              canonical=self.canonical, starts_only=self.starts_only)
        h = torch.from_numpy(np.asarray(hist, dtype=np.int64)).to("cpu" if self.stage_host else self.dev)
        gathered = [torch.empty_like(h) for _ in range(self.world)]
        dist.all_gather(gathered, h, group=self.group)
        H = torch.stack(gathered).cpu().numpy()
        bounds = split_buckets(H.sum(axis=0), self.world)
        self.bucket_bounds = bounds
        b0, b1 = bounds[self.rank], bounds[self.rank + 1]
        mine = np.asarray(hist, dtype=np.int64)
        send_counts = [int(mine[bounds[r]:bounds[r + 1]].sum()) for r in range(self.world)]
        recv_counts = [int(H[s, b0:b1].sum()) for s in range(self.world)]
        R = sum(recv_counts)
        self._ensure_recv(R)
        if not self.starts_only:
            self._exchange(self.send_k, self.recv_k, send_counts, recv_counts)
        self._exchange(self.send_v, self.recv_v, send_counts, recv_counts)
        off, ln, bk = receive_pieces(H, b0, b1, recv_counts)
        if self.recv_v.is_cuda:  # the engine works on its own stream: the exchange must be done
            torch.cuda.current_stream(self.dev).synchronize()
        self.engine.shard_sort(None if self.starts_only else self.recv_k, self.recv_v, R, self.k, off, ln, bk,
                               canonical=self.canonical, starts_only=self.starts_only)
        self.local_kmers = R
        self.engine.materialize_keys()
        return self.engine.unique_count_only()


class KeyRangeKmerSort:
    """One rank of the N-GPU sort with NO data exchange (the default multi-GPU path).

    Every rank already holds the whole sequence byte array -- 1 byte per k-mer, against the
    ~12 bytes per k-mer the all-to-all of ``ShardedKmerSort`` moves over xGMI.  So instead of
    moving k-mers to their owner, each rank re-derives its own from the sequence:

    1. ``shard_histogram``: top-digit histogram of the k-mers starting in the rank's position share;
       on a mixed sba (N runs, IUPAC letters) also ``shard_class_b``: the share's class-B k-mers
       (some non-ACGT letter) as short host lists -- non-homopolymer starts and homopolymer runs --
       with their ownership digits added to the histogram;
    2. ``all_reduce`` (sum) of the 4096-digit histograms -- 32 KiB -- and the same split of the
       digits into N contiguous ranges of about n/N k-mers on every rank (``split_buckets``); on a
       mixed sba an ``all_gather`` of the class-B lists (runs keep them small: GRCh38's N runs are
       ~100 runs, not 150 M starts);
    3. ``shard_sort_range`` / ``shard_sort_range_b``: the rank scans the whole sequence for its
       ACGT-only k-mers (compacted per wave before ranking, so the kept share sets the cost), keeps
       the gathered class-B k-mers of its interval, and sorts them.

    Rank r's sorted k-mers are the r-th slice of the single-GPU order (``Kmers.sort``,
    kmers.py:1624-1652, with break_ties=True, kmers.py:1710-1711): digit ranges ascend with the
    rank, and within a range the sort is the single-GPU sort restricted to it.
    """

    def __init__(self, sba: np.ndarray, seg_starts: np.ndarray, k: int, rank: int, world: int, device: int = 0,
                 engine=None, torch_device=None, group=None, canonical: bool = False):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.group = torch, dist, group
        self.rank, self.world, self.k = rank, world, k
        self.canonical = canonical
        self.dev = torch_device if torch_device is not None else torch.device("cuda", device)
        if engine is None:
            from genome_kmers import _native

            engine = _native.Engine(device)
        self.engine = engine
        t0 = time.perf_counter()
        self.engine.set_sequence(sba, seg_starts)
        self.engine.sync()
        self.h2d_ms = (time.perf_counter() - t0) * 1e3
        bounds = position_ranges(len(sba), world)
        self.lo, self.hi = bounds[rank], bounds[rank + 1]
        self.total_kmers = count_kmers(len(sba), seg_starts, k)
        self.local_kmers = 0
        self.digit_bounds = None

    def _gather_class_b(self, rest: np.ndarray, runs: np.ndarray):
        """all_gather of every rank's class-B lists; concatenated in rank order = start order."""
        torch, dist = self.torch, self.dist
        sizes = torch.tensor([len(rest), len(runs)], dtype=torch.int64, device=self.dev)
        every = [torch.zeros_like(sizes) for _ in range(self.world)]
        dist.all_gather(every, sizes, group=self.group)
        every = [(int(t[0]), int(t[1])) for t in (e.cpu() for e in every)]
        width = max(1, max(a + 3 * b for a, b in every))
        mine = np.zeros(width, dtype=np.uint32)
        mine[:len(rest)] = rest
        mine[len(rest):len(rest) + runs.size] = runs.reshape(-1)
        buf = torch.from_numpy(mine.view(np.int32)).to(self.dev)
        out = [torch.empty_like(buf) for _ in range(self.world)]
        dist.all_gather(out, buf, group=self.group)
        got = [o.cpu().numpy().view(np.uint32) for o in out]
        rest_all = np.concatenate([g[:a] for g, (a, b) in zip(got, every)])
        runs_all = np.concatenate([g[a:a + 3 * b] for g, (a, b) in zip(got, every)]).reshape(-1, 3)
        return rest_all, runs_all

    def run(self) -> int:
        """One sort; returns this rank's number of distinct k-mers."""
        torch, dist = self.torch, self.dist
        hist, bits = self.engine.shard_histogram(self.lo, self.hi, self.k, canonical=self.canonical)
        hist = np.asarray(hist, dtype=np.uint64)
        mixed = not self.engine.is_acgt() and self.k >= 4  # the same on every rank (same sba)
        if mixed:
            rest, runs = self.engine.shard_class_b(self.lo, self.hi, self.k, hist, canonical=self.canonical)
        h = torch.from_numpy(hist.astype(np.int64)).to(self.dev)
        dist.all_reduce(h, group=self.group)
        bounds = split_buckets(h.cpu().numpy(), self.world)
        self.digit_bounds = bounds
        if mixed:
            rest_all, runs_all = self._gather_class_b(rest, runs)
            self.local_kmers = self.engine.shard_sort_range_b(self.k, bounds[self.rank], bounds[self.rank + 1],
                                                              rest_all, runs_all, canonical=self.canonical)
        else:
            self.local_kmers = self.engine.shard_sort_range(self.k, bounds[self.rank], bounds[self.rank + 1],
                                                            canonical=self.canonical)
        self.engine.materialize_keys()  # sorted keys + unique starts and counts stay in HBM
        return self.engine.unique_count_only()
