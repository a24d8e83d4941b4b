"""Config-scale output checks on the GPU -- TEST INFRASTRUCTURE ONLY (PyTorch on the device).

At BASELINE.json's full sizes (3.1e9 k-mers) the CPU oracle cannot sort the input, so the sorted
output of libgkm is checked through size-independent properties, computed here with plain torch
ops on the same GPU, independently of the kernels under test:

* keys are recomputed from the sequence, not taken from the sort: ``position_keys`` builds the key
  of EVERY sequence position by streaming (contiguous shifted slices of a code array, no gather),
  in the reference's byte order (compare_sba_kmers_lexicographically, kmers.py:306-397: raw ASCII
  bytes, '$' below every letter); canonical k-mers take the smaller of forward and reverse
  complement under the reference's complement table (sequence_collection.py:402-433);
* the sorted starts are walked in chunks: the recomputed key of every sorted start must be
  non-decreasing, equal keys must have ascending starts (break_ties=True, kmers.py:1710-1711),
  the product's own keys (if asked) must equal the recomputed ones, every enumerated start
  (kmers.py:789-861: each position with k bases before '$' / the end) must appear exactly once
  (a device bitmap), and the group sizes give the group-size histogram and unique count to
  compare with the product's group pass (kmers.py:454-520).

Device memory is read through the engine's device views with hipMemcpy (the HIP runtime that
torch and libgkm share, genome_kmers._native._share_hip_runtime), chunk by chunk.
"""

from __future__ import annotations

import ctypes
from pathlib import Path

import numpy as np
import torch

DOLLAR = 36
_MIN64 = -(1 << 63)
_hip = None


def hip():
    global _hip
    if _hip is None:
        import importlib.util

        spec = importlib.util.find_spec("torch")
        for root in spec.submodule_search_locations:
            p = Path(root) / "lib" / "libamdhip64.so"
            if p.exists():
                _hip = ctypes.CDLL(str(p))
                break
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipMemcpy.restype = ctypes.c_int
    return _hip


def d2d(dst: torch.Tensor, src_ptr: int, nbytes: int):
    """hipMemcpy device -> device (kind 3) into a torch tensor."""
    if nbytes == 0:
        return
    rc = hip().hipMemcpy(dst.data_ptr(), src_ptr, nbytes, 3)
    assert rc == 0, f"hipMemcpy failed ({rc})"


def _luts(dev):
    c2 = np.zeros(256, dtype=np.int64)
    for ch, v in zip(b"ACGT", range(4)):
        c2[ch] = v
    c4 = np.zeros(256, dtype=np.int64)
    for v, ch in enumerate(b"ABCDGHKMNRSTVWY", start=1):
        c4[ch] = v
    comp = np.arange(256, dtype=np.uint8)
    for a, b in zip(b"ACGTRYSWKMBDHVN$", b"TGCAYRSWMKVHDBN$"):
        comp[a] = b
    return (torch.from_numpy(c2).to(dev), torch.from_numpy(c4).to(dev), torch.from_numpy(comp).to(dev))


class SortedOutputCheck:
    """Recompute keys of every position of a resident sba copy, then walk a sorted output."""

    def __init__(self, sba: np.ndarray, k: int, bits: int, canonical: bool = False, device: str = "cuda"):
        self.dev = torch.device(device)
        self.L = int(sba.size)
        self.k, self.bits, self.canonical = k, bits, canonical
        self.words = (bits * k + 63) // 64
        pad = np.full(self.L + k + 64, DOLLAR, dtype=np.uint8)
        pad[: self.L] = sba
        self.sba = torch.from_numpy(pad).to(self.dev)
        self.c2, self.c4, self.comp = _luts(self.dev)

    # ------------------------------------------------------------------------------------------
    def valid_starts(self) -> torch.Tensor:
        """bool[L]: p is an enumerated k-mer start (no '$' in [p, p + k), p + k <= L)."""
        dol = (self.sba == DOLLAR).to(torch.int32)
        cum = torch.zeros(self.L + self.k + 65, dtype=torch.int32, device=self.dev)
        torch.cumsum(dol, 0, out=cum[1:])
        p = self.L
        return (cum[self.k: self.k + p] - cum[:p]) == 0

    def _words_of(self, codes: torch.Tensor, m: int, reverse: bool):
        """Key words (LSW first) of positions 0..m-1 of `codes` (int64 symbol codes with halo):
        symbol t of the k-mer at p is codes[p + t] (or codes[p + k - 1 - t] if reverse)."""
        k, bits = self.k, self.bits
        lsw = [torch.zeros(m, dtype=torch.int64, device=self.dev) for _ in range(self.words)]
        for t in range(k):
            src = codes[k - 1 - t: k - 1 - t + m] if reverse else codes[t: t + m]
            off = bits * (k - 1 - t)
            w, sh = divmod(off, 64)
            lsw[w] |= src << sh
            if sh + bits > 64:
                lsw[w + 1] |= src >> (64 - sh)
        return lsw[::-1]  # most significant word first

    def position_keys(self, chunk: int = 1 << 27):
        """Per word (most significant first): int64[L] key of the k-mer at every position, sign
        flipped so that signed order = unsigned key order.  Invalid positions hold junk."""
        out = [torch.empty(self.L, dtype=torch.int64, device=self.dev) for _ in range(self.words)]
        lut = self.c2 if self.bits == 2 else self.c4
        for a in range(0, self.L, chunk):
            m = min(chunk, self.L - a)
            raw = self.sba[a: a + m + self.k]
            fw = self._words_of(lut[raw.long()], m, False)
            if self.canonical:
                rc = self._words_of(lut[self.comp[raw.long()].long()], m, True)
                fw = [w ^ _MIN64 for w in fw]
                rc = [w ^ _MIN64 for w in rc]
                lt = torch.zeros(m, dtype=torch.bool, device=self.dev)
                eq = torch.ones(m, dtype=torch.bool, device=self.dev)
                for f, r in zip(fw, rc):
                    lt |= eq & (r < f)
                    eq &= r == f
                for w in range(self.words):
                    out[w][a: a + m] = torch.where(lt, rc[w], fw[w])
            else:
                for w in range(self.words):
                    out[w][a: a + m] = fw[w] ^ _MIN64
            del raw, fw
        return out

    def _word_of(self, codes: torch.Tensor, m: int, reverse: bool, w: int):
        """Key word w (most significant first) of positions 0..m-1, from the symbols that land in it."""
        k, bits = self.k, self.bits
        lw = self.words - 1 - w  # LSW-first index
        out = torch.zeros(m, dtype=torch.int64, device=self.dev)
        for t in range(k):
            off = bits * (k - 1 - t)
            q, sh = divmod(off, 64)
            if q != lw and not (q + 1 == lw and sh + bits > 64):
                continue
            src = codes[k - 1 - t: k - 1 - t + m] if reverse else codes[t: t + m]
            out |= (src << sh) if q == lw else (src >> (64 - sh))
        return out

    def _orientation(self, chunk: int):
        """canonical: uint8[L], 1 where the reverse complement is the smaller k-mer (all words compared)."""
        orient = torch.zeros(self.L, dtype=torch.uint8, device=self.dev)
        lut = self.c2 if self.bits == 2 else self.c4
        for a in range(0, self.L, chunk):
            m = min(chunk, self.L - a)
            raw = self.sba[a: a + m + self.k]
            fw = self._words_of(lut[raw.long()], m, False)
            rc = self._words_of(lut[self.comp[raw.long()].long()], m, True)
            lt = torch.zeros(m, dtype=torch.bool, device=self.dev)
            eq = torch.ones(m, dtype=torch.bool, device=self.dev)
            for f, r in zip(fw, rc):
                f, r = f ^ _MIN64, r ^ _MIN64
                lt |= eq & (r < f)
                eq &= r == f
            orient[a: a + m] = lt.to(torch.uint8)
            del raw, fw, rc
        return orient

    def position_word(self, w: int, orient, chunk: int = 1 << 27):
        """int64[L]: key word w of the k-mer at every position (sign flipped: signed order = unsigned)."""
        out = torch.empty(self.L, dtype=torch.int64, device=self.dev)
        lut = self.c2 if self.bits == 2 else self.c4
        for a in range(0, self.L, chunk):
            m = min(chunk, self.L - a)
            raw = self.sba[a: a + m + self.k]
            f = self._word_of(lut[raw.long()], m, False, w)
            if orient is not None:
                r = self._word_of(lut[self.comp[raw.long()].long()], m, True, w)
                f = torch.where(orient[a: a + m].bool(), r, f)
            out[a: a + m] = f ^ _MIN64
            del raw, f
        return out

    def check_sorted_wordwise(self, starts_ptr, n: int, keys_ptr=0, key_words: int = 0,
                              max_counts_bin: int = 64, chunk: int = 1 << 27, unique=None):
        """check_sorted for keys too large to recompute whole (C5: 4 words x 3.09 G k-mers = 99 GB
        beside the product's own 99 GB): ONE word of every position's key at a time (25 GB), the
        canonical orientation of every position decided first over all words (1 B each).  Each
        word pass compares the product's word with the recomputed one and advances a per-pair
        state (0 equal so far, 1 ordered, 2 out of order); a last pass over the sorted starts
        checks tie order, group heads, multiplicities, the histogram and the permutation."""
        ubuf = torch.empty(chunk + 1, dtype=torch.int32, device=self.dev)

        def read_u32(src, a, m):
            if isinstance(src, np.ndarray):
                ubuf[:m] = torch.from_numpy(src[a:a + m].astype(np.uint32).view(np.int32))
            else:
                d2d(ubuf, src + 4 * a, 4 * m)
            return ubuf[:m].to(torch.int64) & 0xFFFFFFFF

        s32 = torch.empty(chunk + 1, dtype=torch.int32, device=self.dev)

        def starts(a, m):
            if isinstance(starts_ptr, np.ndarray):
                s32[:m] = torch.from_numpy(starts_ptr[a:a + m].view(np.int32))
            else:
                d2d(s32, starts_ptr + 4 * a, 4 * m)
            return s32[:m].to(torch.int64) & 0xFFFFFFFF

        orient = self._orientation(chunk) if self.canonical else None
        state = torch.zeros(max(n - 1, 0), dtype=torch.uint8, device=self.dev)  # pair (i - 1, i) at i - 1
        kbuf = torch.empty(chunk, dtype=torch.int64, device=self.dev)
        for w in range(self.words):
            pw = self.position_word(w, orient, chunk)
            prev = None
            for a in range(0, n, chunk):
                m = min(chunk, n - a)
                g = pw[starts(a, m)]
                if isinstance(keys_ptr, np.ndarray) or keys_ptr:
                    assert key_words == self.words
                    if isinstance(keys_ptr, np.ndarray):
                        kbuf[:m] = torch.from_numpy(keys_ptr[a:a + m, w].view(np.int64))
                    else:
                        d2d(kbuf, keys_ptr + 8 * (w * n + a), 8 * m)
                    assert torch.equal(kbuf[:m] ^ _MIN64, g), f"product key word {w} differs in [{a}, {a + m})"
                gg = g if prev is None else torch.cat([prev.view(1), g])
                lo = a if prev is None else a - 1  # first pair index covered
                st = state[lo: lo + gg.numel() - 1]
                und = st == 0
                st[und & (gg[1:] < gg[:-1])] = 2
                st[und & (gg[1:] > gg[:-1])] = 1
                prev = g[-1].clone()
                del g, gg
            del pw
            torch.cuda.empty_cache() if self.dev.type == "cuda" else None
        assert not bool((state == 2).any().item()), "keys out of order"
        del orient
        valid = self.valid_starts()
        n_valid = int(valid.sum().item())
        assert n == n_valid, f"{n} sorted starts but {n_valid} enumerated k-mers"
        seen = torch.zeros(self.L, dtype=torch.uint8, device=self.dev)
        hist = torch.zeros(max_counts_bin + 1, dtype=torch.int64, device=self.dev)
        prev_start, last_head, groups = None, 0, 0
        for a in range(0, n, chunk):
            m = min(chunk, n - a)
            s = starts(a, m)
            assert int(s.max().item()) < self.L, "start index out of range"
            assert bool(valid[s].all().item()), "a sorted start is not an enumerated k-mer start"
            seen[s] = 1
            if prev_start is not None:
                s = torch.cat([prev_start.view(1), s])
            base = a if prev_start is None else a - 1
            eq = state[base: base + s.numel() - 1] == 0
            assert bool((s[1:][eq] > s[:-1][eq]).all().item()), f"equal k-mers not in start order near {a}"
            heads = torch.nonzero(~eq).flatten() + base + 1
            if prev_start is None:
                heads = torch.cat([torch.zeros(1, dtype=torch.int64, device=self.dev), heads])
            if unique is not None and heads.numel():
                assert groups + heads.numel() <= unique[2], "fewer unique k-mers in the product than groups"
                got = read_u32(unique[0], groups, heads.numel())
                assert torch.equal(got, heads), f"product group starts differ from the groups near {a}"
            if heads.numel():
                bounds = torch.cat([torch.tensor([last_head], device=self.dev), heads])
                sizes = bounds[1:] - bounds[:-1]
                if prev_start is None:
                    sizes = sizes[1:]
                hist += torch.bincount(sizes.clamp(max=max_counts_bin), minlength=max_counts_bin + 1)
                groups += heads.numel()
                last_head = int(heads[-1].item())
            prev_start = s[-1].clone()
        if n:
            hist[min(n - last_head, max_counts_bin)] += 1
        if unique is not None:
            G = unique[2]
            assert G == groups, f"product has {G} unique k-mers, the sorted order {groups} groups"
            total = 0
            for a in range(0, G, chunk):
                m = min(chunk, G - a)
                gs = read_u32(unique[0], a, m).clone()
                nxt = read_u32(unique[0], a + 1, m - 1) if m > 1 else gs[:0]
                end = n if a + m >= G else int(read_u32(unique[0], a + m, 1)[0].item())
                want = torch.cat([nxt, torch.tensor([end], device=self.dev)]) - gs
                cnt = read_u32(unique[1], a, m)
                assert torch.equal(cnt, want), f"product multiplicities differ near unique k-mer {a}"
                total += int(cnt.sum().item())
            assert total == n, "multiplicities do not sum to the number of k-mers"
        assert torch.equal(seen.bool(), valid), "sorted starts are not a permutation of the enumerated starts"
        del seen, valid, state
        if self.dev.type == "cuda":
            torch.cuda.empty_cache()
        return groups, hist.cpu().numpy()

    # ------------------------------------------------------------------------------------------
    def check_sorted(self, starts_ptr, n: int, keys_ptr=0, key_words: int = 0,
                     max_counts_bin: int = 64, chunk: int = 1 << 27, unique=None):
        """Walk n sorted starts (device uint32 at starts_ptr, or a host uint32 array) and the
        product's keys (device uint64 SoA at keys_ptr, or a host (n, words) array; 0 = none).
        unique = (group_start, count, n_unique) of the product's unique output (device uint32
        pointers or host arrays): every group start must be a recomputed group head, and every
        count the distance to the next head.
        Returns (n_groups, hist) and asserts order, tie order, permutation and keys."""
        ubuf = torch.empty(chunk + 1, dtype=torch.int32, device=self.dev)

        def read_u32(src, a, m):
            if isinstance(src, np.ndarray):
                ubuf[:m] = torch.from_numpy(src[a:a + m].astype(np.uint32).view(np.int32))
            else:
                d2d(ubuf, src + 4 * a, 4 * m)
            return ubuf[:m].to(torch.int64) & 0xFFFFFFFF
        pk = self.position_keys()
        valid = self.valid_starts()
        n_valid = int(valid.sum().item())
        assert n == n_valid, f"{n} sorted starts but {n_valid} enumerated k-mers"
        seen = torch.zeros(self.L, dtype=torch.uint8, device=self.dev)
        s32 = torch.empty(chunk, dtype=torch.int32, device=self.dev)
        kbuf = torch.empty(chunk, dtype=torch.int64, device=self.dev)
        hist = torch.zeros(max_counts_bin + 1, dtype=torch.int64, device=self.dev)
        prev_key, prev_start = None, None
        last_head, groups = 0, 0
        for a in range(0, n, chunk):
            m = min(chunk, n - a)
            if isinstance(starts_ptr, np.ndarray):
                s32[:m] = torch.from_numpy(starts_ptr[a:a + m].view(np.int32))
            else:
                d2d(s32, starts_ptr + 4 * a, 4 * m)
            s = s32[:m].to(torch.int64) & 0xFFFFFFFF
            assert int(s.max().item()) < self.L, "start index out of range"
            assert bool(valid[s].all().item()), "a sorted start is not an enumerated k-mer start"
            seen[s] = 1
            g = [w[s] for w in pk]
            if isinstance(keys_ptr, np.ndarray) or keys_ptr:
                assert key_words == self.words
                for w in range(self.words):
                    if isinstance(keys_ptr, np.ndarray):
                        kbuf[:m] = torch.from_numpy(keys_ptr[a:a + m, w].view(np.int64))
                    else:
                        d2d(kbuf, keys_ptr + 8 * (w * n + a), 8 * m)
                    assert torch.equal(kbuf[:m] ^ _MIN64, g[w]), f"product key word {w} differs in [{a}, {a + m})"
            # adjacent pairs inside the chunk, plus the pair across the chunk boundary
            if prev_key is not None:
                g = [torch.cat([pv.view(1), w]) for pv, w in zip(prev_key, g)]
                s = torch.cat([prev_start.view(1), s])
            lt = torch.zeros(s.numel() - 1, dtype=torch.bool, device=self.dev)
            eq = torch.ones(s.numel() - 1, dtype=torch.bool, device=self.dev)
            for w in g:
                lt |= eq & (w[1:] < w[:-1])  # a later key smaller than its predecessor
                eq &= w[1:] == w[:-1]
            assert not bool(lt.any().item()), f"keys out of order near sorted index {a}"
            assert bool((s[1:][eq] > s[:-1][eq]).all().item()), f"equal k-mers not in start order near {a}"
            # group heads (global sorted indices) -> sizes of the groups closed in this chunk
            base = a if prev_key is None else a - 1
            heads = torch.nonzero(~eq).flatten() + base + 1
            if prev_key is None:
                heads = torch.cat([torch.zeros(1, dtype=torch.int64, device=self.dev), heads])
            if unique is not None and heads.numel():
                assert groups + heads.numel() <= unique[2], "fewer unique k-mers in the product than groups"
                got = read_u32(unique[0], groups, heads.numel())
                assert torch.equal(got, heads), f"product group starts differ from the groups near {a}"
            if heads.numel():
                bounds = torch.cat([torch.tensor([last_head], device=self.dev), heads])
                sizes = bounds[1:] - bounds[:-1]
                if prev_key is None:
                    sizes = sizes[1:]  # heads[0] = 0 opens the first group
                hist += torch.bincount(sizes.clamp(max=max_counts_bin), minlength=max_counts_bin + 1)
                groups += heads.numel()
                last_head = int(heads[-1].item())
            prev_key = [w[-1].clone() for w in g]
            prev_start = s[-1].clone()
            del g, s
        if n:
            hist[min(n - last_head, max_counts_bin)] += 1
        if unique is not None:
            G = unique[2]
            assert G == groups, f"product has {G} unique k-mers, the sorted order {groups} groups"
            total = 0
            for a in range(0, G, chunk):
                m = min(chunk, G - a)
                gs = read_u32(unique[0], a, m).clone()
                nxt = read_u32(unique[0], a + 1, m - 1) if m > 1 else gs[:0]
                end = n if a + m >= G else int(read_u32(unique[0], a + m, 1)[0].item())
                want = torch.cat([nxt, torch.tensor([end], device=self.dev)]) - gs
                cnt = read_u32(unique[1], a, m)
                assert torch.equal(cnt, want), f"product multiplicities differ near unique k-mer {a}"
                total += int(cnt.sum().item())
            assert total == n, "multiplicities do not sum to the number of k-mers"
        assert torch.equal(seen.bool(), valid), "sorted starts are not a permutation of the enumerated starts"
        del pk, seen, valid
        torch.cuda.empty_cache()
        return groups, hist.cpu().numpy()


def window_keys(eng, off: int, m: int) -> np.ndarray:
    """(m, words) product keys at sorted offsets [off, off + m), read from the device key array
    (word-major, stride n) word by word with hipMemcpy D2H -- no full-size host copy."""
    _, keys_ptr, n, words = eng.device_views()
    out = np.empty((m, words), dtype=np.uint64)
    tmp = np.empty(m, dtype=np.uint64)
    for q in range(words):
        rc = hip().hipMemcpy(tmp.ctypes.data, keys_ptr + 8 * (q * n + off), 8 * m, 2)
        assert rc == 0, f"hipMemcpy failed ({rc})"
        out[:, q] = tmp
    return out


def oracle_windows(km, sba: np.ndarray, k: int, offsets, width: int = 4096, canonical: bool = False,
                   keys: bool = False):
    """Host windows of the sorted starts at the given sorted offsets, checked with the CPU oracle's
    restatement of the reference comparator (kmers.py:306-397) pair by pair: each window must be
    non-decreasing, with equal k-mers in ascending start order.  keys: the product's keys of the
    window must equal the oracle's keys of its starts (4-bit, or 2-bit on an ACGT-only sba)."""
    from oracle import oracle

    eng = km._engine
    n = eng.n
    for off in offsets:
        off = int(min(max(off, 0), max(n - width, 0)))
        w = eng.start_range(off, min(width, n - off))
        if keys:
            bits = 2 if eng.is_acgt() else 4
            got = window_keys(eng, off, len(w))
            want = (oracle.canonical_keys(sba, w, k, bits) if canonical
                    else oracle.encode_keys(sba, w, *oracle.key_spec(bits == 2, k, k)))
            np.testing.assert_array_equal(got, want.reshape(got.shape), err_msg=f"keys at sorted index {off}")
        if canonical:
            canon, _ = oracle.canonical_windows(sba, w, k)
            for i in range(len(w) - 1):
                a, b = bytes(canon[i]), bytes(canon[i + 1])
                assert a < b or (a == b and w[i] < w[i + 1]), f"canonical order broken at sorted index {off + i}"
        else:
            for i in range(len(w) - 1):
                cmp, _ = oracle.compare(sba, int(w[i]), int(w[i + 1]), k)
                assert cmp < 0 or (cmp == 0 and w[i] < w[i + 1]), f"order broken at sorted index {off + i}"
