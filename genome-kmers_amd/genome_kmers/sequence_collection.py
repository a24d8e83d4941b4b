"""SequenceCollection -- the input contract of the k-mer engine (host side).

Mirrors mrperkett/genome-kmers ``genome_kmers/sequence_collection.py`` (v1.0.1) so that code
written against the reference runs unchanged: the same constructor, members, record iteration,
location lookups, error types and messages.  The sequence byte array (SBA) built here is exactly
the reference's: contigs' ASCII bytes joined by '$' (36), no trailing '$', uint32 segment starts
(sequence_collection.py:531-576, 663-726).  ``Kmers`` uploads it to HBM; this module itself is
host bookkeeping and performs no k-mer work.
"""

import pickle
import shelve
from collections import Counter
from pathlib import Path
from typing import Callable, List, Union

import numpy as np

DOLLAR = ord("$")
_ALLOWED_BASES = {"A", "C", "G", "T", "R", "Y", "S", "W", "K", "M", "B", "D", "H", "V", "N", "$"}
_ALLOWED_UINT8 = {ord(b) for b in _ALLOWED_BASES}
_ALLOWED_LUT = np.zeros(256, dtype=bool)
_ALLOWED_LUT[list(_ALLOWED_UINT8)] = True


def bisect_right(a, x):
    """Insertion point to the right of any x in sorted a (sequence_collection.py:15-39)."""
    return int(np.searchsorted(np.asarray(a), x, side="right"))


def reverse_complement_sba(sba: np.ndarray, complement_mapping_arr: np.ndarray, inplace=False) -> np.ndarray:
    """Reverse complement through a uint8 -> uint8 map (sequence_collection.py:42-73)."""
    rc = complement_mapping_arr[sba[::-1]]
    if inplace:
        sba[:] = rc
        return sba
    return rc.astype(np.uint8)


def get_segment_num_from_sba_index(sba_idx: int, sba_strand: str, sba_seg_starts: np.ndarray) -> int:
    """Segment holding sba_idx (sequence_collection.py:76-97)."""
    return bisect_right(sba_seg_starts, sba_idx) - 1


def get_forward_seq_idx(sba_idx, sba_strand, seg_sba_start_idx, seg_sba_end_idx, one_based=False) -> int:
    """Sequence index of an sba index (sequence_collection.py:100-152)."""
    if sba_idx < seg_sba_start_idx:
        raise ValueError(f"sba_idx ({sba_idx}) must be >= seg_sba_start_idx ({seg_sba_start_idx})")
    if sba_idx > seg_sba_end_idx:
        raise ValueError(f"sba_idx ({sba_idx}) must be <= seg_end_start_idx ({seg_sba_end_idx})")
    if seg_sba_start_idx > seg_sba_end_idx:
        raise ValueError(
            f"seg_sba_start_idx ({seg_sba_start_idx}) must be <= seg_sba_end_idx ({seg_sba_end_idx})"
        )
    if seg_sba_start_idx < 0:
        raise ValueError(f"seg_sba_start_idx ({seg_sba_start_idx}) must be > 0")
    if sba_strand == "forward":
        seq_idx = sba_idx - seg_sba_start_idx
    elif sba_strand == "reverse_complement":
        seq_idx = seg_sba_end_idx - sba_idx
    else:
        raise ValueError(f"sba_strand ({sba_strand}) not recognized")
    return int(seq_idx) + (1 if one_based else 0)


def get_sba_start_end_indices_for_segment(segment_num: int, sba_strand: str, sba_seg_starts: np.ndarray,
                                          len_sba: int) -> tuple:
    """First and last sba index of a segment (sequence_collection.py:155-187)."""
    if segment_num < 0 or segment_num >= len(sba_seg_starts):
        raise ValueError(f"segment_num ({segment_num}) is out of bounds")
    start = int(sba_seg_starts[segment_num])
    if segment_num == len(sba_seg_starts) - 1:
        end = int(len_sba) - 1
    else:
        end = int(sba_seg_starts[segment_num + 1]) - 2
    return start, end


class SequenceCollection:
    """FASTA / sequence-list contents packed as a sequence byte array (see module docstring)."""

    def __init__(self, fasta_file_path: Union[Path, None] = None,
                 sequence_list: Union[list, None] = None, strands_to_load: str = "forward") -> None:
        self.forward_sba = None
        self._forward_sba_seg_starts = None
        self.forward_record_names = None
        self.revcomp_sba = None
        self._revcomp_sba_seg_starts = None
        self.revcomp_record_names = None
        self._strands_loaded = None
        self._fasta_file_path = None
        self._initialize_mapping_arrays()
        if fasta_file_path is None and sequence_list is None:
            return
        if fasta_file_path is not None and sequence_list is not None:
            raise ValueError("Only one of fasta_file_path and sequence_list can be specified")
        if strands_to_load not in ("forward", "reverse_complement", "both"):
            raise ValueError(f"strands_to_load unrecognized ({strands_to_load})")
        if fasta_file_path is not None:
            self._fasta_file_path = fasta_file_path
            self._initialize_from_fasta(fasta_file_path, strands_to_load)
        else:
            self._initialize_from_sequence_list(sequence_list, strands_to_load)

    # -----------------------------------------------------------------------------------------
    def __len__(self) -> int:
        if self._strands_loaded in ("forward", "both"):
            return len(self._forward_sba_seg_starts)
        if self._strands_loaded == "reverse_complement":
            return len(self._revcomp_sba_seg_starts)
        raise AssertionError(f"strands_loaded ({self._strands_loaded}) not recognized")

    def __str__(self) -> str:
        strand = "reverse_complement" if self._strands_loaded == "reverse_complement" else "forward"
        sba = self.forward_sba if strand == "forward" else self.revcomp_sba
        lines = []
        for name, b, e in self.iter_records(strand):
            lines.append(f">{name}")
            lines.append(bytes(sba[b : e + 1]).decode())
        return "\n".join(lines)

    def sequence_length(self, record_num=None, record_name=None):
        if record_name is not None and record_num is not None:
            raise ValueError(
                f"record_num ({record_num}) and record_name ({record_name}) cannot both be specified"
            )
        raise NotImplementedError()

    def iter_records(self, sba_strand: str = None):
        """Yield (record_name, sba_start, sba_end) in record order (sequence_collection.py:356-391)."""
        sba_strand = self._get_sba_strand_to_use(sba_strand)
        if sba_strand == "forward":
            for s in range(len(self)):
                b, e = get_sba_start_end_indices_for_segment(s, sba_strand, self._forward_sba_seg_starts,
                                                             len(self.forward_sba))
                yield (self.forward_record_names[s], b, e)
        elif sba_strand == "reverse_complement":
            for s in range(len(self) - 1, -1, -1):
                b, e = get_sba_start_end_indices_for_segment(s, sba_strand, self._revcomp_sba_seg_starts,
                                                             len(self.revcomp_sba))
                yield (self.revcomp_record_names[s], b, e)
        else:
            raise ValueError(f"sba_strand ({sba_strand}) must be 'forward' or 'reverse_complement'")

    def strands_loaded(self) -> str:
        return self._strands_loaded

    @staticmethod
    def _get_complement_mapping_array():
        pairs = {"A": "T", "C": "G", "G": "C", "T": "A", "R": "Y", "Y": "R", "S": "S", "W": "W", "K": "M",
                 "M": "K", "B": "V", "D": "H", "H": "D", "V": "B", "N": "N", "$": "$"}
        arr = np.zeros(256, dtype=np.uint8)
        for k, v in pairs.items():
            arr[ord(k)] = ord(v)
        return arr

    def _initialize_mapping_arrays(self):
        self._allowed_bases = set(_ALLOWED_BASES)
        self._allowed_uint8 = set(_ALLOWED_UINT8)
        self._complement_mapping_arr = SequenceCollection._get_complement_mapping_array()
        self._uint8_to_u1_mapping = np.array([chr(i) for i in range(256)], dtype="U1")
        self._u1_to_uint8_mapping = {chr(i): i for i in range(256)}
        self._numba_unicode_to_uint8_mapping = {chr(i): np.uint8(i) for i in range(256)}

    # ---- FASTA (sequence_collection.py:476-632) ----------------------------------------------
    @staticmethod
    def _get_fasta_stats(fasta_file_path: Path) -> tuple:
        num_records = 0
        total_seq_len = 0
        with open(fasta_file_path, "r") as fh:
            for line in fh:
                if line.startswith(">"):
                    num_records += 1
                else:
                    total_seq_len += len(line.strip())
        return num_records, total_seq_len

    @staticmethod
    def _get_fasta_record_name(line: str) -> str:
        if not line.startswith(">"):
            raise ValueError("line does not start with '>'")
        return line[1:].strip().split()[0]

    def _check_alphabet(self, sba: np.ndarray):
        if sba.size and not _ALLOWED_LUT[sba].all():
            bad = set(np.unique(sba[~_ALLOWED_LUT[sba]]).tolist())
            raise ValueError(f"Sequence contains non-allowed characters! ({bad})")

    def _load_forward_sba_from_fasta(self, fasta_file_path: Path, num_records: int = None, total_seq_len: int = None):
        """The reference's per-line loop (sequence_collection.py:517-576) as libgkm's multithreaded
        host parser (gkm_fasta.cpp: memory-mapped, chunked at line starts, one scan + one parallel
        fill); same bytes, then the reference's checks in its order."""
        from genome_kmers import _native

        try:
            sba, seg_starts, names, bad = _native.read_fasta(fasta_file_path)
        except _native.FastaLayoutError:
            raise AssertionError("After parsing the fasta file, we expect sba to be full") from None
        if (np.diff(seg_starts.astype(np.int64)) < 2).any():
            raise ValueError(f"At least one empty sequence was found in the input file ({fasta_file_path})")
        SequenceCollection._verify_record_names_are_unique(names)
        if bad:
            raise ValueError(f"Sequence contains non-allowed characters! ({bad})")
        return sba, seg_starts, names

    def _initialize_from_fasta(self, fasta_file_path: Path, strands_to_load: str) -> None:
        if strands_to_load not in ("forward", "reverse_complement", "both"):
            raise ValueError(f"strands_to_load not recognized ({strands_to_load})")
        self.forward_sba, self._forward_sba_seg_starts, self.forward_record_names = (
            self._load_forward_sba_from_fasta(fasta_file_path)
        )
        self._strands_loaded = "forward"
        self._finish_strands(strands_to_load)

    # ---- sequence list (sequence_collection.py:634-819) --------------------------------------
    @staticmethod
    def _get_required_sba_length_from_sequence_list(sequence_list) -> int:
        total = 0
        for name, seq in sequence_list:
            if len(seq) == 0:
                raise ValueError(
                    f"Each sequence in the collection must have length > 0.  Record '{name}' has a sequence lengt of 0"
                )
            total += len(seq)
        return total + len(sequence_list) - 1

    def _get_sba_from_sequence_list(self, sequence_list) -> np.ndarray:
        n = SequenceCollection._get_required_sba_length_from_sequence_list(sequence_list)
        sba = np.zeros(n, dtype=np.uint8)
        at = 0
        for i, (_, seq) in enumerate(sequence_list):
            b = seq.encode("utf-8") if isinstance(seq, str) else bytes(seq)
            sba[at : at + len(b)] = np.frombuffer(b, dtype=np.uint8)
            at += len(b)
            if i != len(sequence_list) - 1:
                sba[at] = DOLLAR
                at += 1
        self._check_alphabet(sba)
        return sba

    @staticmethod
    def _get_sba_starts_from_sequence_list(sequence_list) -> np.ndarray:
        starts = np.zeros(len(sequence_list), dtype=np.uint32)
        at = 0
        for i, (_, seq) in enumerate(sequence_list):
            starts[i] = at
            at += len(seq) + 1
        return starts

    @staticmethod
    def _verify_record_names_are_unique(record_names):
        counter = Counter(record_names)
        if len(record_names) != len(counter):
            repeated = len([1 for c in counter.values() if c > 1])
            raise ValueError(f"sequence_list contains {repeated} repeated record_names")

    @staticmethod
    def _get_record_names_from_sequence_list(sequence_list) -> List[str]:
        names = [name for name, _ in sequence_list]
        SequenceCollection._verify_record_names_are_unique(names)
        return names

    def _initialize_from_sequence_list(self, sequence_list, strands_to_load: str):
        if strands_to_load not in ("forward", "reverse_complement", "both"):
            raise ValueError(f"strands_to_load not recognized ({strands_to_load})")
        self.forward_sba = self._get_sba_from_sequence_list(sequence_list)
        self._forward_sba_seg_starts = self._get_sba_starts_from_sequence_list(sequence_list)
        self.forward_record_names = self._get_record_names_from_sequence_list(sequence_list)
        self._strands_loaded = "forward"
        self._finish_strands(strands_to_load)

    def _finish_strands(self, strands_to_load: str):
        if strands_to_load == "both":
            self.revcomp_sba = reverse_complement_sba(self.forward_sba, self._complement_mapping_arr)
            self._revcomp_sba_seg_starts = self._get_opposite_strand_sba_start_indices(
                self._forward_sba_seg_starts, len(self.revcomp_sba))
            self.revcomp_record_names = list(reversed(self.forward_record_names))
            self._strands_loaded = "both"
        elif strands_to_load == "reverse_complement":
            self.reverse_complement()

    # ---- strands (sequence_collection.py:821-928) --------------------------------------------
    def reverse_complement(self) -> None:
        if self._strands_loaded == "both":
            raise ValueError(f"self._strands_loaded ({self._strands_loaded}) cannot be 'both'")
        if self._strands_loaded == "forward":
            self.revcomp_sba = reverse_complement_sba(self.forward_sba, self._complement_mapping_arr, inplace=True)
            self.forward_sba = None
            self._revcomp_sba_seg_starts = self._get_opposite_strand_sba_start_indices(
                self._forward_sba_seg_starts, len(self.revcomp_sba))
            self._forward_sba_seg_starts = None
            self.revcomp_record_names = self.forward_record_names
            self.revcomp_record_names.reverse()
            self.forward_record_names = None
            self._strands_loaded = "reverse_complement"
        elif self._strands_loaded == "reverse_complement":
            self.forward_sba = reverse_complement_sba(self.revcomp_sba, self._complement_mapping_arr, inplace=True)
            self.revcomp_sba = None
            self._forward_sba_seg_starts = self._get_opposite_strand_sba_start_indices(
                self._revcomp_sba_seg_starts, len(self.forward_sba))
            self._revcomp_sba_seg_starts = None
            self.forward_record_names = self.revcomp_record_names
            self.forward_record_names.reverse()
            self.revcomp_record_names = None
            self._strands_loaded = "forward"

    @staticmethod
    def _get_opposite_strand_sba_index(sba_idx: int, sba_len: int) -> int:
        if sba_idx < 0 or sba_idx >= sba_len:
            raise ValueError(f"sba_idx ({sba_idx}) is out of bounds")
        return sba_len - 1 - sba_idx

    @staticmethod
    def _get_opposite_strand_sba_indices(sba_indices: np.ndarray, sba_len: int) -> np.ndarray:
        if (sba_indices < 0).any() or (sba_indices >= sba_len).any():
            raise ValueError("There is at least one sba index that is out of bounds")
        return sba_len - 1 - sba_indices

    @staticmethod
    def _get_opposite_strand_sba_start_indices(sba_starts: np.ndarray, sba_len: int) -> np.ndarray:
        ends = np.copy(sba_starts)
        if len(ends) > 1:
            ends[:-1] = ends[1:] - 2
        ends[-1] = sba_len - 1
        return SequenceCollection._get_opposite_strand_sba_indices(np.flip(ends), sba_len)

    # ---- location lookups (sequence_collection.py:930-1187) ----------------------------------
    def _strand_arrays(self, sba_strand):
        if sba_strand == "forward":
            return self.forward_sba, self._forward_sba_seg_starts, self.forward_record_names
        return self.revcomp_sba, self._revcomp_sba_seg_starts, self.revcomp_record_names

    def get_record_loc_from_sba_index(self, sba_idx: int, sba_strand: str = None, one_based: bool = False) -> tuple:
        sba_strand = self._get_sba_strand_to_use(sba_strand)
        if sba_strand not in ("forward", "reverse_complement"):
            raise ValueError(f"sba_strand ({sba_strand}) not recognized")
        sba, starts, names = self._strand_arrays(sba_strand)
        seg = get_segment_num_from_sba_index(sba_idx, sba_strand, starts)
        b, e = get_sba_start_end_indices_for_segment(seg, sba_strand, starts, len(sba))
        seq_idx = get_forward_seq_idx(sba_idx, sba_strand, b, e, one_based=one_based)
        return ("+" if sba_strand == "forward" else "-", names[seg], seq_idx)

    def get_record_name_from_sba_index(self, sba_idx: int, sba_strand: str = None) -> str:
        sba_strand = self._get_sba_strand_to_use(sba_strand)
        if sba_strand not in ("forward", "reverse_complement"):
            raise ValueError(f"sba_strand ({sba_strand}) not recognized")
        _, starts, names = self._strand_arrays(sba_strand)
        return names[get_segment_num_from_sba_index(sba_idx, sba_strand, starts)]

    def _get_sba_strand_to_use(self, sba_strand: str) -> str:
        if sba_strand is not None:
            if sba_strand == "forward":
                if self._strands_loaded == "reverse_complement":
                    raise ValueError(
                        f"sba_strand ({sba_strand}) does not match _strands_loaded ({self._strands_loaded})"
                    )
            elif sba_strand == "reverse_complement":
                if self._strands_loaded == "forward":
                    raise ValueError(
                        f"sba_strand ({sba_strand}) does not match _strands_loaded ({self._strands_loaded})"
                    )
            else:
                raise ValueError(f"sba_strand ({sba_strand}) not recognized")
        if self._strands_loaded == "both" and sba_strand is None:
            raise ValueError("sba_strand must be specified when both strands are loaded")
        return self._strands_loaded if self._strands_loaded != "both" else sba_strand

    def get_segment_num_from_sba_index(self, sba_idx: int, sba_strand: str = None) -> int:
        sba_strand = self._get_sba_strand_to_use(sba_strand)
        sba, starts, _ = self._strand_arrays(sba_strand)
        if sba_idx < 0 or sba_idx >= len(sba):
            raise IndexError(f"sba_idx ({sba_idx}) is out of bounds")
        return get_segment_num_from_sba_index(sba_idx, sba_strand, starts)

    def get_sba_start_end_indices_for_segment(self, segment_num: int, sba_strand: str = None) -> tuple:
        sba_strand = self._get_sba_strand_to_use(sba_strand)
        sba, starts, _ = self._strand_arrays(sba_strand)
        return get_sba_start_end_indices_for_segment(segment_num, sba_strand, starts, len(sba))

    def generate_get_record_info_from_sba_index_func(self, one_based: bool = False) -> Callable:
        sba_strand = self._get_sba_strand_to_use(self.strands_loaded())
        if sba_strand not in ("forward", "reverse_complement"):
            raise ValueError(f"sba_strand ({sba_strand}) not recognized")
        sba, starts, names = self._strand_arrays(sba_strand)
        names = tuple(names)
        strand_char = "+" if sba_strand == "forward" else "-"
        len_sba = len(sba)

        def get_record_info_from_sba_index(sba_idx: int) -> tuple:
            seg = get_segment_num_from_sba_index(sba_idx, sba_strand, starts)
            b, e = get_sba_start_end_indices_for_segment(seg, sba_strand, starts, len_sba)
            seq_idx = get_forward_seq_idx(sba_idx, sba_strand, b, e, one_based=one_based)
            return (seg, b, e, strand_char, names[seg], seq_idx)

        return get_record_info_from_sba_index

    # ---- equality / persistence (sequence_collection.py:1189-1446) ---------------------------
    def __ne__(self, other):
        return not self.__eq__(other)

    def __eq__(self, other):
        for attr in ("forward_sba", "_forward_sba_seg_starts", "revcomp_sba", "_revcomp_sba_seg_starts"):
            a, b = getattr(self, attr), getattr(other, attr)
            if (a is None) != (b is None):
                return False
            if a is not None and not np.array_equal(a, b):
                return False
        for attr in ("forward_record_names", "revcomp_record_names", "_strands_loaded"):
            a, b = getattr(self, attr), getattr(other, attr)
            if (a is None) != (b is None):
                return False
            if a is not None and a != b:
                return False
        return True

    def save(self, save_file_path: Path, mode: str = "a", format: str = "hdf5") -> None:
        if format == "hdf5":
            self._save_hdf5(save_file_path, mode=mode)
        elif format == "shelve":
            self._save_shelve(save_file_path)
        else:
            raise ValueError(f"format ({format}) not recognized")

    def load(self, load_file_path: Path, format: str = "hdf5"):
        if format == "hdf5":
            self._load_h5py(load_file_path)
        elif format == "shelve":
            self._load_shelve(load_file_path)
        else:
            raise ValueError(f"format ({format}) not recognized")

    def _save_hdf5(self, save_file_path: Path, mode: str = "a") -> None:
        import h5py  # optional dependency, as in the reference

        def ex(v, empty):
            return empty if v is None else v

        with h5py.File(save_file_path, mode) as f:
            g = f.create_group("seq_coll")
            g["forward_sba"] = ex(self.forward_sba, np.array([], dtype=np.uint8))
            g["_forward_sba_seg_starts"] = ex(self._forward_sba_seg_starts, [])
            g["forward_record_names"] = ex(self.forward_record_names, [])
            g["revcomp_sba"] = ex(self.revcomp_sba, np.array([], dtype=np.uint8))
            g["_revcomp_sba_seg_starts"] = ex(self._revcomp_sba_seg_starts, [])
            g["revcomp_record_names"] = ex(self.revcomp_record_names, [])
            g["_strands_loaded"] = ex(self._strands_loaded, "")
            g["_fasta_file_path"] = str(ex(self._fasta_file_path, ""))

    def _load_h5py(self, load_file_path: Path):
        import h5py

        def im(v):
            if isinstance(v, np.ndarray):
                return None if v.shape == (0,) else v
            return None if v in ("", []) else v

        with h5py.File(load_file_path, "r") as f:
            g = f["seq_coll"]
            self.forward_sba = im(g["forward_sba"][:])
            self._forward_sba_seg_starts = im(g["_forward_sba_seg_starts"][:])
            self.forward_record_names = im([v.decode("utf-8") for v in g["forward_record_names"]])
            self.revcomp_sba = im(g["revcomp_sba"][:])
            self._revcomp_sba_seg_starts = im(g["_revcomp_sba_seg_starts"][:])
            self.revcomp_record_names = im([v.decode("utf-8") for v in g["revcomp_record_names"]])
            self._strands_loaded = im(g["_strands_loaded"][()].decode("utf-8"))
            fp = im(g["_fasta_file_path"][()].decode("utf-8"))
            self._fasta_file_path = Path(fp) if fp is not None else None
        self._initialize_mapping_arrays()

    def _save_shelve(self, save_file_path: Path) -> None:
        with shelve.open(str(save_file_path), protocol=pickle.DEFAULT_PROTOCOL) as db:
            for k in ("forward_sba", "_forward_sba_seg_starts", "forward_record_names", "revcomp_sba",
                      "_revcomp_sba_seg_starts", "revcomp_record_names", "_strands_loaded", "_fasta_file_path"):
                db[f"seq_coll.{k}"] = getattr(self, k)

    def _load_shelve(self, load_file_path: Path):
        with shelve.open(str(load_file_path)) as db:
            for k in ("forward_sba", "_forward_sba_seg_starts", "forward_record_names", "revcomp_sba",
                      "_revcomp_sba_seg_starts", "revcomp_record_names", "_strands_loaded", "_fasta_file_path"):
                setattr(self, k, db[f"seq_coll.{k}"])
        self._initialize_mapping_arrays()
