"""Synthetic genomes of BASELINE.json's configs, shared by bench.py and the
config-scale parity tests.  There is no network and no FASTA on the GPU box, so every config is a
seeded surrogate of stated shape.  C3 is the reference's own profiling genome:
``profiling.get_random_seq`` after ``np.random.seed(seed)`` (``np.random.choice`` over
``["A", "T", "G", "C"]``, profiling.py:12-24), made by libgkm's host MT19937
(``gk_reference_random_bases``: the same bytes as numpy's legacy RandomState, 3.1 Gb in seconds
and without a 25 GB int64 temporary).  The other surrogates use numpy's PCG64 in chunks.

Every function returns ``(sba, seg_starts)`` in the reference's SequenceCollection layout
(contigs joined by '$', no trailing '$'; sequence_collection.py:663-726).
"""

from __future__ import annotations

import numpy as np

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
_CHUNK = 1 << 28

# GRCh38 primary assembly chromosome lengths, chr1..chr22, chrX, chrY (total 3,088,269,832 bp)
GRCH38_LENGTHS = [248956422, 242193529, 198295559, 190214555, 181538259, 170805979, 159345973, 145138636,
                  138394717, 133797422, 135086622, 133275309, 114364328, 107043718, 101991189, 90338345,
                  83257441, 80373285, 58617616, 64444167, 46709983, 50818468, 156040895, 57227415]

C2_LENGTH = 4_641_652  # E. coli K-12 MG1655


def random_bases(L: int, seed: int, lut: np.ndarray = np.frombuffer(b"ATGC", dtype=np.uint8)) -> np.ndarray:
    """L uniform i.i.d. bases (the reference's alphabet order b"ATGC", profiling.py:12-24)."""
    out = np.empty(L, dtype=np.uint8)
    rng = np.random.default_rng(seed)
    for at in range(0, L, _CHUNK):
        m = min(_CHUNK, L - at)
        out[at:at + m] = lut[rng.integers(0, 4, m, dtype=np.uint8)]
    return out


def c3_genome(L: int = 3_100_000_000, seed: int = 42):
    """C3: one random contig of L bases (BASELINE.json configs[2]) -- the reference's profiling
    genome for this seed (profiling.get_random_seq(L) after np.random.seed(seed))."""
    from genome_kmers import _native

    return _native.reference_random_bases(L, seed), np.zeros(1, dtype=np.uint32)


def c2_surrogate(seed: int = 1, L: int = C2_LENGTH):
    """C2 without the E. coli FASTA: one contig of E. coli K-12's length, uniform random ACGT, with
    the genome's two repeat classes planted so that tie groups exist -- 7 copies of one 5 kb
    "rRNA operon" and 10 copies of one 1.3 kb "IS element", exact copies at random positions."""
    rng = np.random.default_rng(seed)
    sba = ACGT[rng.integers(0, 4, L, dtype=np.uint8)]
    for unit_len, copies in ((5000, 7), (1300, 10)):
        unit = ACGT[rng.integers(0, 4, unit_len, dtype=np.uint8)]
        for at in rng.integers(0, L - unit_len, copies):
            sba[at:at + unit_len] = unit
    return sba, np.zeros(1, dtype=np.uint32)


def grch38_surrogate(seed: int = 2, lengths=GRCH38_LENGTHS):
    """C4/C5 input without a FASTA: GRCh38's 24 contig lengths joined by '$', uniform random ACGT,
    ~5 % N (runs at both contig ends and the centre), and repeat families with realistic divergence
    so that k-mer groups of every size exist:
      Alu-like  300 bp x 400,000 copies, 12 % substitutions;  L1-like 6 kb x 15,000 copies, 8 %;
      segmental duplications 20 kb x 300 exact copies;  (CA)n microsatellites 40 bp x 50,000.
    ``lengths`` may be scaled down for tests (every feature keeps its per-contig proportion;
    repeat copy numbers scale with the total length)."""
    rng = np.random.default_rng(seed)
    L = int(sum(lengths)) + len(lengths) - 1
    scale = L / (sum(GRCH38_LENGTHS) + len(GRCH38_LENGTHS) - 1)
    sba = np.empty(L, dtype=np.uint8)
    for at in range(0, L, _CHUNK):
        m = min(_CHUNK, L - at)
        sba[at:at + m] = ACGT[rng.integers(0, 4, m, dtype=np.uint8)]

    def plant(unit, copies, div):
        copies = max(1, int(round(copies * scale)))
        if L <= len(unit):
            return
        at = rng.integers(0, L - len(unit), copies)
        for a in range(0, copies, 20_000):
            b = min(copies, a + 20_000)
            rows = np.broadcast_to(unit, (b - a, len(unit))).copy()
            mut = rng.random(rows.shape) < div
            rows[mut] = ACGT[rng.integers(0, 4, int(mut.sum()), dtype=np.uint8)]
            sba[at[a:b, None] + np.arange(len(unit))[None, :]] = rows

    plant(ACGT[rng.integers(0, 4, 300)], 400_000, 0.12)
    plant(ACGT[rng.integers(0, 4, 6000)], 15_000, 0.08)
    for _ in range(max(1, int(round(300 * scale)))):
        if L <= 40_000:
            break
        src, dst = rng.integers(0, L - 20_000, 2)
        sba[dst:dst + 20_000] = sba[src:src + 20_000]
    plant(np.frombuffer(b"CA" * 20, dtype=np.uint8), 50_000, 0.0)
    starts = np.concatenate([[0], np.cumsum(np.asarray(lengths[:-1], dtype=np.int64) + 1)])
    for s0, n in zip(starts, lengths):
        e, c = int(n * 0.015), int(n * 0.02)
        sba[s0:s0 + e] = ord("N")
        sba[s0 + n - e:s0 + n] = ord("N")
        sba[s0 + n // 2 - c // 2:s0 + n // 2 + c // 2] = ord("N")
    sba[starts[1:] - 1] = ord("$")
    return sba, starts.astype(np.uint32)
