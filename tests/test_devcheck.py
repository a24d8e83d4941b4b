"""The config-scale checker (tests/devcheck.py) on the CPU: it accepts the oracle's sorted output
and rejects every kind of corruption it is meant to catch (order, tie order, duplicates, missing
starts, wrong keys, wrong group sizes), so a green full-size GPU test means something."""

import numpy as np
import pytest

import devcheck
from oracle import oracle


def _case(k=9, canonical=False, seed=3):
    rng = np.random.default_rng(seed)
    sba = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, 3000)].copy()
    sba[1000:1200] = sba[100:300]              # repeats: tie groups
    sba[2000] = ord("$")                        # two contigs
    sba[2500:2520] = ord("N")                   # N run (4-bit keys)
    seg = np.array([0, 2001], dtype=np.uint32)
    starts = oracle.enumerate_starts(sba, seg, k)
    if canonical:
        srt = oracle.canonical_sort(sba, starts, k)
        keys = oracle.canonical_keys(sba, srt, k, 4)
        hist, _ = oracle.canonical_group_hist(sba, srt, k, max_counts_bin=8)
    else:
        srt = oracle.quicksort(sba, starts, k, k, break_ties=True)
        keys = oracle.encode_keys(sba, srt, 4, k, 0, (4 * k + 63) // 64)
        hist, _ = oracle.group_scan(sba, srt, k, max_counts_bin=8)
    return sba, srt, keys, hist


@pytest.mark.parametrize("k,canonical", [(9, False), (20, False), (9, True), (17, True)])
def test_accepts_oracle_output(k, canonical):
    sba, srt, keys, hist = _case(k, canonical)
    chk = devcheck.SortedOutputCheck(sba, k, 4, canonical=canonical, device="cpu")
    gs, cnt = _unique(keys)
    groups, h = chk.check_sorted(srt, len(srt), keys_ptr=keys, key_words=keys.shape[1], max_counts_bin=8,
                                 chunk=257, unique=(gs, cnt, len(gs)))
    np.testing.assert_array_equal(h, hist)
    assert groups == int(hist.sum())


def _unique(keys):
    heads = np.concatenate([[True], (keys[1:] != keys[:-1]).any(axis=1)])
    gs = np.flatnonzero(heads).astype(np.uint32)
    cnt = np.diff(np.append(gs.astype(np.int64), len(keys))).astype(np.uint32)
    return gs, cnt


def test_rejects_wrong_multiplicity():
    sba, srt, keys, _ = _case()
    gs, cnt = _unique(keys)
    i = int(np.argmax(cnt > 1))
    cnt = cnt.copy()
    cnt[i] -= 1
    chk = devcheck.SortedOutputCheck(sba, 9, 4, device="cpu")
    with pytest.raises(AssertionError, match="multiplicities"):
        chk.check_sorted(srt, len(srt), keys_ptr=keys, key_words=keys.shape[1], max_counts_bin=8, chunk=257,
                         unique=(gs, cnt, len(gs)))


def test_rejects_wrong_group_start():
    sba, srt, keys, _ = _case()
    gs, cnt = _unique(keys)
    gs = gs.copy()
    gs[300] += 1
    chk = devcheck.SortedOutputCheck(sba, 9, 4, device="cpu")
    with pytest.raises(AssertionError, match="group starts"):
        chk.check_sorted(srt, len(srt), keys_ptr=keys, key_words=keys.shape[1], max_counts_bin=8, chunk=257,
                         unique=(gs, cnt, len(gs)))


def _expect_fail(sba, srt, keys, k=9, match=None):
    chk = devcheck.SortedOutputCheck(sba, k, 4, device="cpu")
    with pytest.raises(AssertionError, match=match):
        chk.check_sorted(srt, len(srt), keys_ptr=keys, key_words=keys.shape[1], max_counts_bin=8, chunk=257)


def test_rejects_swapped_keys():
    sba, srt, keys, _ = _case()
    i = 700
    while keys[i, 0] == keys[i + 1, 0]:
        i += 1
    srt = srt.copy()
    srt[[i, i + 1]] = srt[[i + 1, i]]
    keys = keys.copy()
    keys[[i, i + 1]] = keys[[i + 1, i]]
    _expect_fail(sba, srt, keys, match="out of order")


def test_rejects_swapped_ties():
    sba, srt, keys, _ = _case()
    ties = np.flatnonzero(keys[1:, 0] == keys[:-1, 0])
    i = int(ties[len(ties) // 2])
    srt = srt.copy()
    srt[[i, i + 1]] = srt[[i + 1, i]]
    _expect_fail(sba, srt, keys, match="start order")


def test_rejects_duplicate_start():
    sba, srt, keys, _ = _case()
    srt = srt.copy()
    ties = np.flatnonzero(keys[1:, 0] == keys[:-1, 0])
    i = int(ties[0])
    srt[i + 1] = srt[i]  # a k-mer counted twice, another lost
    _expect_fail(sba, srt, keys)


def test_rejects_wrong_product_key():
    sba, srt, keys, _ = _case()
    keys = keys.copy()
    keys[1234, 0] ^= 1
    _expect_fail(sba, srt, keys, match="product key")


def test_rejects_missing_kmer():
    sba, srt, keys, _ = _case()
    _expect_fail(sba, srt[:-1], keys[:-1], match="enumerated")


# the word-wise checker (multi-word keys at full size, devcheck.check_sorted_wordwise)
@pytest.mark.parametrize("k,canonical", [(9, False), (20, False), (9, True), (17, True), (33, True)])
def test_wordwise_accepts_oracle_output(k, canonical):
    sba, srt, keys, hist = _case(k, canonical)
    chk = devcheck.SortedOutputCheck(sba, k, 4, canonical=canonical, device="cpu")
    gs, cnt = _unique(keys)
    groups, h = chk.check_sorted_wordwise(srt, len(srt), keys_ptr=keys, key_words=keys.shape[1], max_counts_bin=8,
                                          chunk=257, unique=(gs, cnt, len(gs)))
    np.testing.assert_array_equal(h, hist)
    assert groups == int(hist.sum())


@pytest.mark.parametrize("what", ["key", "order", "ties", "dup", "mult"])
def test_wordwise_rejects(what):
    sba, srt, keys, _ = _case(20, True)
    gs, cnt = _unique(keys)
    srt, keys, cnt = srt.copy(), keys.copy(), cnt.copy()
    if what == "key":
        keys[500, 1] ^= 1
        match = "product key word 1"
    elif what == "order":  # two distinct neighbours swapped, keys with them
        i = int(np.flatnonzero((keys[1:] != keys[:-1]).any(axis=1))[10])
        srt[[i, i + 1]] = srt[[i + 1, i]]
        keys[[i, i + 1]] = keys[[i + 1, i]]
        match = "out of order"
    elif what == "ties":  # two members of a tie group swapped
        i = int(np.flatnonzero((keys[1:] == keys[:-1]).all(axis=1))[0])
        srt[[i, i + 1]] = srt[[i + 1, i]]
        match = "start order"
    elif what == "dup":
        srt[10] = srt[11]
        keys[10] = keys[11]
        match = None
    else:
        cnt[int(np.argmax(cnt > 1))] -= 1
        match = "multiplicities"
    chk = devcheck.SortedOutputCheck(sba, 20, 4, canonical=True, device="cpu")
    with pytest.raises(AssertionError, match=match):
        chk.check_sorted_wordwise(srt, len(srt), keys_ptr=keys, key_words=keys.shape[1], max_counts_bin=8,
                                  chunk=257, unique=(gs, cnt, len(gs)))
