"""FASTA ingest: libgkm's multithreaded host parser (gk_fasta_open /
gk_fasta_fill, genome-kmers_amd/csrc/gkm_fasta.cpp) behind SequenceCollection(fasta_file_path=...)
against the reference loader restated in oracle/fasta.py (sequence_collection.py:476-576).

The inputs of the reference's own TestFastaInit (test_sequence_collection.py:300-500) are replayed
from real files here (the reference mocks ``open``; a native parser reads the file itself), plus
the edge cases of Python's text-mode line handling, and multi-chunk parses (GKM_FASTA_CHUNK) whose
chunk edges fall inside lines, inside '\\r\\n' pairs and on headers.  Host only: no GPU.
"""

import numpy as np
import pytest

from genome_kmers import _native
from genome_kmers.sequence_collection import SequenceCollection
from oracle import fasta as ofasta

# the reference's fixtures (test_sequence_collection.py:35-50, 318-335)
FASTA_1 = ">chr1\nATCGAATTAG"
FASTA_2 = ">chr1\nATCGAATTAG\n>chr2\nGGATCTTGCATT\n>chr3\nGTGATTGACCCCT"
EMPTY_SEQ = ">chr1\nATGC\n>chr2\n\n>chr3\nATGC"
ILLEGAL = ">chr1\nATGC+"
REPEATED = ">chr1\nATGC\n>chr1\nATGC"


def _write(tmp_path, data, name="x.fa"):
    p = tmp_path / name
    p.write_bytes(data.encode() if isinstance(data, str) else data)
    return p


def _outcome(fn):
    try:
        return ("ok", fn())
    except Exception as e:  # noqa: BLE001 -- the exception type and message are the contract
        return (type(e).__name__, str(e))


def _check_same(path):
    want = _outcome(lambda: ofasta.load_fasta(path))
    got = _outcome(lambda: SequenceCollection(fasta_file_path=path, strands_to_load="forward"))
    assert got[0] == want[0], (got, want)
    if want[0] == "ok":
        sba, starts, names = want[1]
        sc = got[1]
        np.testing.assert_array_equal(sc.forward_sba, sba)
        np.testing.assert_array_equal(sc._forward_sba_seg_starts, starts)
        assert sc.forward_record_names == names
        assert sc.forward_sba.dtype == np.uint8 and sc._forward_sba_seg_starts.dtype == np.uint32
    else:
        assert got[1] == want[1]
    return got


def test_reference_fixture_single_record(tmp_path):
    sc = _check_same(_write(tmp_path, FASTA_1))[1]
    assert bytes(sc.forward_sba) == b"ATCGAATTAG"
    assert sc.forward_record_names == ["chr1"]
    assert sc._forward_sba_seg_starts.tolist() == [0]


def test_reference_fixture_three_records(tmp_path):
    sc = _check_same(_write(tmp_path, FASTA_2))[1]
    assert bytes(sc.forward_sba) == b"ATCGAATTAG$GGATCTTGCATT$GTGATTGACCCCT"
    assert sc._forward_sba_seg_starts.tolist() == [0, 11, 24]
    assert str(sc) == FASTA_2


@pytest.mark.parametrize("strands", ["reverse_complement", "both"])
def test_reference_fixture_strands(tmp_path, strands):
    p = _write(tmp_path, FASTA_2)
    sc = SequenceCollection(fasta_file_path=p, strands_to_load=strands)
    ref = SequenceCollection(sequence_list=[("chr1", "ATCGAATTAG"), ("chr2", "GGATCTTGCATT"),
                                            ("chr3", "GTGATTGACCCCT")], strands_to_load=strands)
    assert sc == ref


@pytest.mark.parametrize("data,exc", [(EMPTY_SEQ, ValueError), (ILLEGAL, ValueError), (REPEATED, ValueError)])
def test_reference_fixture_errors(tmp_path, data, exc):
    p = _write(tmp_path, data)
    with pytest.raises(exc):
        SequenceCollection(fasta_file_path=p, strands_to_load="forward")
    _check_same(p)


EDGE = {
    "crlf": ">a\r\nACGT\r\nAC\r\n>b\r\nGG\r\n",
    "lone_cr": ">a\rACGT\rAC\r>b\rGG",
    "mixed_endings": ">a\nAC\r\nGT\rTT\n>b\r\nC",
    "lowercase": ">a\nacgtn\nACgtRyswkm\n",
    "whitespace": ">a  desc here\n  ACGT \t\nAC\x0b\x0c\n\n\n>\tb\tx\n GG \n",
    "py_space_1c_1f": ">a\n\x1cAC\x1f\n>b\nG\x1dG\x1e\n",
    "blank_lines": "\n\n>a\n\nAC\n\n>b\nG\n\n",
    "last_record_empty": ">a\nACGT\n>b\n",
    "first_record_empty": ">a\n>b\nACGT\n",
    "no_trailing_newline": ">a\nACGT\n>b\nTTT",
    "iupac": ">a\nACGTRYSWKMBDHVN\n>b\nnnnnACGT\n",
    "dollar_inside": ">a\nAC$GT\n",
    "header_no_name": ">a\nAC\n>\nGG\n",
    "header_space_only": ">a\nAC\n>   \nGG\n",
    "space_before_gt": ">a\nAC\n >b\nGG\n",
    "bad_chars": ">a\nACXGT\n>b\nAC-.*\n",
    "long_lines": ">a\n" + "ACGT" * 5000 + "\n>b\n" + "T" * 12345 + "\n",
}


@pytest.mark.parametrize("name", sorted(EDGE))
def test_edge_cases_match_reference_loader(tmp_path, name):
    _check_same(_write(tmp_path, EDGE[name]))


def test_empty_file_raises_like_reference(tmp_path):
    p = _write(tmp_path, "")
    with pytest.raises(ValueError):
        ofasta.load_fasta(p)
    with pytest.raises(ValueError):
        SequenceCollection(fasta_file_path=p, strands_to_load="forward")


def test_sequence_before_first_header_raises(tmp_path):
    # the reference fails inside its copy (numpy broadcast / index error); the native parser
    # reports the sba it cannot fill exactly (AssertionError, sequence_collection.py:565-566)
    p = _write(tmp_path, "ACGT\n>a\nGG\n")
    with pytest.raises(Exception):
        ofasta.load_fasta(p)
    with pytest.raises(AssertionError):
        SequenceCollection(fasta_file_path=p, strands_to_load="forward")


def test_missing_file(tmp_path):
    with pytest.raises(FileNotFoundError):
        SequenceCollection(fasta_file_path=tmp_path / "nope.fa", strands_to_load="forward")


def _random_fasta(rng, nrec, line_len, ending="\n"):
    parts = []
    for r in range(nrec):
        parts.append(f">rec{r} some description{ending}")
        L = int(rng.integers(1, 20_000))
        seq = rng.choice(np.frombuffer(b"ACGTacgtNnRY", dtype=np.uint8), L).tobytes().decode()
        for i in range(0, L, line_len):
            parts.append(seq[i:i + line_len] + ending)
        if rng.random() < 0.2:
            parts.append(ending)
    return "".join(parts)


@pytest.mark.parametrize("chunk,ending,seed", [(7, "\n", 1), (64, "\r\n", 2), (4093, "\n", 3), (1, "\r\n", 4),
                                              (100_000, "\r", 5)])
def test_multichunk_parse_matches_reference(tmp_path, monkeypatch, chunk, ending, seed):
    rng = np.random.default_rng(seed)
    p = _write(tmp_path, _random_fasta(rng, 40 if chunk > 1 else 6, int(rng.integers(50, 90)), ending))
    monkeypatch.setenv("GKM_FASTA_CHUNK", str(chunk))
    _check_same(p)


def test_read_fasta_thread_counts_agree(tmp_path, monkeypatch):
    rng = np.random.default_rng(9)
    p = _write(tmp_path, _random_fasta(rng, 30, 61))
    monkeypatch.setenv("GKM_FASTA_CHUNK", "997")
    outs = [_native.read_fasta(p, n_threads=t) for t in (1, 3, 16)]
    for sba, starts, names, bad in outs[1:]:
        np.testing.assert_array_equal(sba, outs[0][0])
        np.testing.assert_array_equal(starts, outs[0][1])
        assert names == outs[0][2] and bad == outs[0][3]
