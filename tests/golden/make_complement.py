"""Golden vectors for the reverse-complement mapping, produced by the reference itself.

Test infrastructure, run once in the build container like make_golden.py (same identity-JIT numba
stub; nothing of the reference is copied).  It records:
  complement_lut      SequenceCollection._get_complement_mapping_array()  (sequence_collection.py:402-433)
  sba / rc_sba        an IUPAC multi-record forward sba and reverse_complement_sba(sba, lut)
                      (sequence_collection.py:42-73)
  both_sba            SequenceCollection(strands_to_load="both").revcomp_sba of the same records
The canonical k-mer order of the device path (min of a k-mer and its reverse complement) is
built on this mapping; tests/test_oracle_golden.py pins the oracle's mapping to these vectors.

Run:  /opt/conda/bin/python3.9 tests/golden/make_complement.py
"""

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden  # noqa: E402  (sets up the reference import path and the numba stub)
from genome_kmers.sequence_collection import SequenceCollection, reverse_complement_sba  # noqa: E402


def main():
    rng = np.random.default_rng(5)
    alphabet = np.frombuffer(b"ACGTRYSWKMBDHVN", dtype=np.uint8)
    records = [(f"r{i}", rng.choice(alphabet, n).tobytes().decode()) for i, n in enumerate([700, 1, 64, 333])]
    fwd = SequenceCollection(sequence_list=records, strands_to_load="forward")
    lut = SequenceCollection._get_complement_mapping_array()
    rc = reverse_complement_sba(fwd.forward_sba, lut)
    both = SequenceCollection(sequence_list=records, strands_to_load="both")
    np.savez_compressed(os.path.join(make_golden.OUT_DIR, "complement.npz"), complement_lut=lut,
                        sba=fwd.forward_sba, rc_sba=rc, both_sba=both.revcomp_sba)
    print("complement.npz:", len(fwd.forward_sba), "bytes")


if __name__ == "__main__":
    main()
