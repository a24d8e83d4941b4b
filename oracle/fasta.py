"""Reference FASTA loader restated in pure Python -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` import this module (as the checker of libgkm's gk_fasta_open / gk_fasta_fill);
the product never does.

Follows sequence_collection.py line for line in behaviour:
  _get_fasta_stats                :476-515  (records, sum of len(line.strip()) over sequence lines)
  _get_fasta_record_name          :578-586  (line[1:].strip().split()[0])
  _load_forward_sba_from_fasta    :517-576  (text mode = universal newlines; '$' unless at == 0;
                                             .strip().upper(); the at == sba_len assertion; the
                                             empty-record, unique-name and alphabet checks)
Returns (sba, seg_starts, names) or raises what the reference raises.
"""

from collections import Counter

import numpy as np

DOLLAR = ord("$")
ALLOWED = np.zeros(256, dtype=bool)
ALLOWED[[ord(c) for c in "ACGTRYSWKMBDHVN$"]] = True


def fasta_stats(path):
    num_records = 0
    total_seq_len = 0
    with open(path, "r") as fh:
        for line in fh:
            if line.startswith(">"):
                num_records += 1
            else:
                total_seq_len += len(line.strip())
    return num_records, total_seq_len


def record_name(line):
    if not line.startswith(">"):
        raise ValueError("line does not start with '>'")
    return line[1:].strip().split()[0]


def load_fasta(path):
    num_records, total_seq_len = fasta_stats(path)
    sba_len = total_seq_len + num_records - 1
    seg_starts = np.zeros(num_records, dtype=np.uint32)
    sba = np.zeros(sba_len, dtype=np.uint8)
    names = []
    at = 0
    rec = -1
    with open(path, "r") as fh:
        for line in fh:
            if line.startswith(">"):
                rec += 1
                if at != 0:
                    sba[at] = DOLLAR
                    at += 1
                seg_starts[rec] = at
                names.append(record_name(line))
            else:
                chunk = np.frombuffer(line.strip().upper().encode("utf-8"), dtype=np.uint8)
                sba[at : at + chunk.size] = chunk
                at += chunk.size
    if at != sba_len:
        raise AssertionError("After parsing the fasta file, we expect sba to be full")
    if (np.diff(seg_starts.astype(np.int64)) < 2).any():
        raise ValueError(f"At least one empty sequence was found in the input file ({path})")
    counter = Counter(names)  # _verify_record_names_are_unique (sequence_collection.py:749-759)
    if len(names) != len(counter):
        repeated = len([1 for c in counter.values() if c > 1])
        raise ValueError(f"sequence_list contains {repeated} repeated record_names")
    if sba.size and not ALLOWED[sba].all():
        bad = set(np.unique(sba[~ALLOWED[sba]]).tolist())
        raise ValueError(f"Sequence contains non-allowed characters! ({bad})")
    return sba, seg_starts, names
