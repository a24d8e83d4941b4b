"""Generate reference-pinned CONTRACT fixtures by running the reference genome-kmers itself.

Test infrastructure, run ONCE in the build container (the reference is at /root/reference, read
only; numba's JIT replaced by the identity stub of make_golden.py).  Only data is committed:
``contracts.json`` plus the HDF5 files the reference's own ``save`` wrote (``persist_*.h5``).

Sections of contracts.json:
  kmers_init        Kmers.__init__ argument checks: exception type + message, or the enumerated
                    starts (kmers.py:656-760; the reference's TestInit, test_kmers.py:250-470)
  seqcoll_init      SequenceCollection argument / alphabet / record checks (sequence_collection.py:
                    200-320, 441-458, 663-726; test_sequence_collection.py:82-275)
  fasta             SequenceCollection(fasta_file_path=...) on the reference's TestFastaInit inputs
                    and on text-mode edge cases: sba, segment starts, record names, or the error
                    (sequence_collection.py:476-576)
  full_info         Kmers.get_kmers(kmer_info_to_yield="full") on the stable (break_ties=True) order
                    (kmers.py:869-992, 1180-1264)
  persistence       Kmers.save / load in both formats (kmers.py:1306-1531, sequence_collection.py:
                    1293-1446): the HDF5 layout the reference writes and the state it loads back

Run:  /opt/conda/bin/python3.9 tests/golden/make_contracts.py
"""

import base64
import json
import os
import shelve
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (installs the numba stub + the reference on sys.path)

import h5py  # noqa: E402

gk, SequenceCollection = mg.gk, mg.SequenceCollection

SEQ_LIST_1 = [("chr1", "ATCGAATTAG")]
SEQ_LIST_2 = mg.SEQ_LIST_2


def outcome(fn):
    try:
        return {"ok": fn()}
    except Exception as e:  # noqa: BLE001 -- the type and message are the contract
        return {"error": type(e).__name__, "message": str(e)}


# ---------------------------------------------------------------------------------------------
def kmers_init_cases():
    sc1 = lambda: SequenceCollection(sequence_list=SEQ_LIST_1, strands_to_load="forward")  # noqa: E731
    sc2 = lambda: SequenceCollection(sequence_list=SEQ_LIST_2, strands_to_load="forward")  # noqa: E731

    def rc1():
        s = sc1()
        s.reverse_complement()
        return s

    colls = {"seq_list_1": sc1, "seq_list_2": sc2, "seq_list_1_revcomp": rc1}
    kw = [
        {"min_kmer_len": 0},
        {"min_kmer_len": -3},
        {"min_kmer_len": 100},
        {"min_kmer_len": 10},
        {"min_kmer_len": 11},
        {"min_kmer_len": 1, "max_kmer_len": 0},
        {"min_kmer_len": 5, "max_kmer_len": 4},
        {"min_kmer_len": 2, "max_kmer_len": 1000},
        {"min_kmer_len": 3, "max_kmer_len": 3},
        {},
        {"source_strand": "reverse_complement"},
        {"source_strand": "both"},
        {"source_strand": "bogus"},
        {"track_strands_separately": True},
        {"source_strand": "both", "track_strands_separately": True},
        {"method": "double_pass"},
        {"method": "bogus"},
        {"min_kmer_len": 0, "max_kmer_len": 0},
        {"min_kmer_len": 4, "max_kmer_len": 2, "source_strand": "bogus"},
    ]
    out = []
    for cname, make in colls.items():
        for k in kw:
            def run():
                km = gk.Kmers(make(), **k)
                return km.kmer_sba_start_indices.tolist()
            out.append({"collection": cname, "kwargs": k, "result": outcome(run)})
    # an empty SequenceCollection object (no records)
    out.append({"collection": "empty", "kwargs": {}, "result": outcome(lambda: gk.Kmers(SequenceCollection()))})
    return out


def seqcoll_init_cases():
    cases = [
        {"sequence_list": SEQ_LIST_1, "strands_to_load": "something_incorrect"},
        {"sequence_list": [("chr1", "ATCGAATTA.")]},
        {"sequence_list": [("chr1", "")]},
        {"sequence_list": [("chr1", "ATCGAATTA"), ("chr2", ""), ("chr3", "AAAATGC")]},
        {"sequence_list": [("chr1", "ATCGAATTA"), ("chr1", "AAAATGC")]},
        {"sequence_list": [("chr1", "acgtn")]},
        {"sequence_list": [("chr1", "ACGT$ACGT")]},
        {"sequence_list": [("chr1", "ACGTRYSWKMBDHVN")]},
        {"sequence_list": [("chr1", "ACGU")]},
        {"sequence_list": SEQ_LIST_2, "strands_to_load": "reverse_complement"},
        {"sequence_list": SEQ_LIST_2, "strands_to_load": "both"},
    ]
    out = []
    for c in cases:
        args = dict(c)
        args.setdefault("strands_to_load", "forward")

        def run():
            sc = SequenceCollection(**args)
            return {"forward_sba": None if sc.forward_sba is None else bytes(sc.forward_sba).decode("latin-1"),
                    "seg_starts": None if sc._forward_sba_seg_starts is None else sc._forward_sba_seg_starts.tolist(),
                    "names": sc.forward_record_names, "strands": sc.strands_loaded()}
        out.append({"args": {k: (v if k != "sequence_list" else [list(t) for t in v]) for k, v in args.items()},
                    "result": outcome(run)})
    out.append({"args": {"fasta_file_path": "x.fa", "sequence_list": [["chr1", "ACGT"]],
                         "strands_to_load": "forward"},
                "result": outcome(lambda: SequenceCollection(fasta_file_path="x.fa", sequence_list=SEQ_LIST_1,
                                                             strands_to_load="forward"))})
    return out


# the reference's TestFastaInit inputs (test_sequence_collection.py:35-50, 318-335) and text-mode
# edge cases of Python's line handling
FASTA_INPUTS = {
    "ref_fasta_1": ">chr1\nATCGAATTAG",
    "ref_fasta_2": ">chr1\nATCGAATTAG\n>chr2\nGGATCTTGCATT\n>chr3\nGTGATTGACCCCT",
    "ref_empty_sequence": ">chr1\nATGC\n>chr2\n\n>chr3\nATGC",
    "ref_illegal_base": ">chr1\nATGC+",
    "ref_repeated_name": ">chr1\nATGC\n>chr1\nATGC",
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
    "header_space_only": ">a\nAC\n>   \nGG\n",
    "space_before_gt": ">a\nAC\n >b\nGG\n",
    "bad_chars": ">a\nACXGT\n>b\nAC-.*\n",
    "multi_line_80col": ">chrA desc\n" + "\n".join(["ACGTTGCA" * 10] * 7) + "\nACG\n>chrB\n" + "\n".join(["TTGGCCAA" * 10] * 3),
    "long_lines": ">a\n" + "ACGT" * 5000 + "\n>b\n" + "T" * 12345 + "\n",
}


def random_fasta(seed, nrec, line_len, ending="\n"):
    rng = np.random.default_rng(seed)
    parts = []
    for r in range(nrec):
        parts.append(f">rec{r} some description{ending}")
        L = int(rng.integers(1, 3000))
        seq = rng.choice(np.frombuffer(b"ACGTacgtNnRY", dtype=np.uint8), L).tobytes().decode()
        for i in range(0, L, line_len):
            parts.append(seq[i:i + line_len] + ending)
        if rng.random() < 0.2:
            parts.append(ending)
    return "".join(parts)


def fasta_cases():
    inputs = dict(FASTA_INPUTS)
    for seed, ending in ((1, "\n"), (2, "\r\n"), (3, "\r")):
        inputs[f"random_{seed}"] = random_fasta(seed, 12, 61 + seed, ending)
    out = []
    tmp = tempfile.mkdtemp(prefix="gk_fasta_")
    for name, data in inputs.items():
        path = os.path.join(tmp, f"{name}.fa")
        with open(path, "wb") as fh:
            fh.write(data.encode("latin-1"))

        def run():
            sc = SequenceCollection(fasta_file_path=path, strands_to_load="forward")
            return {"forward_sba": bytes(sc.forward_sba).decode("latin-1"),
                    "seg_starts": sc._forward_sba_seg_starts.tolist(), "names": sc.forward_record_names}
        res = outcome(run)
        if "message" in res:  # the file's path appears in some messages
            res["message"] = res["message"].replace(path, "{path}")
        out.append({"name": name, "data_b64": base64.b64encode(data.encode("latin-1")).decode(), "result": res})
    return out


# ---------------------------------------------------------------------------------------------
def full_info_cases():
    genomes = {
        "seq_list_2": SEQ_LIST_2,
        "iupac_small": [(n, s[:700]) for n, s in mg.iupac_genome(11) if len(s) >= 700],
        "repeat": mg.repeat_genome(5),
    }
    queries = [
        {"kmer_len": None, "one_based": False, "yield_first_n": None, "min_group_size": 1, "max_group_size": None},
        {"kmer_len": 3, "one_based": False, "yield_first_n": None, "min_group_size": 1, "max_group_size": None},
        {"kmer_len": 3, "one_based": True, "yield_first_n": 2, "min_group_size": 2, "max_group_size": None},
        {"kmer_len": 5, "one_based": True, "yield_first_n": None, "min_group_size": 1, "max_group_size": 3},
        {"kmer_len": 8, "one_based": False, "yield_first_n": 1, "min_group_size": 2, "max_group_size": None},
        {"kmer_len": 12, "one_based": True, "yield_first_n": 3, "min_group_size": 1, "max_group_size": None},
    ]
    out = []
    for gname, seqs in genomes.items():
        for mn, mx in ((3, None), (3, 12), (5, 5)):
            sc = SequenceCollection(sequence_list=seqs, strands_to_load="forward")
            km = gk.Kmers(sc, min_kmer_len=mn, max_kmer_len=mx)
            km.kmer_sba_start_indices = mg.stable_sort(km)
            km._is_sorted = True
            for qi, qy in enumerate(queries):
                if gname != "seq_list_2" and qi in (0, 1):
                    continue  # every k-mer of a 2-4 kb genome: kept to the grouped queries
                kl = qy["kmer_len"]
                if kl is not None and (kl < mn or (mx is not None and kl > mx)):
                    continue

                def run():
                    rows = km.get_kmers(kl, kmer_info_to_yield="full", one_based_seq_index=qy["one_based"],
                                        min_group_size=qy["min_group_size"], max_group_size=qy["max_group_size"],
                                        yield_first_n=qy["yield_first_n"])
                    return [[int(x) if isinstance(x, (int, np.integer)) else x for x in r] for r in rows]
                out.append({"genome": gname, "min_kmer_len": mn, "max_kmer_len": mx, "query": qy,
                            "result": outcome(run)})
    return out


def h5_layout(path):
    lay = {}

    def visit(name, obj):
        if isinstance(obj, h5py.Dataset):
            v = obj[()]
            if isinstance(v, bytes):
                val = {"bytes": v.decode("latin-1")}
            elif isinstance(v, np.ndarray):
                val = [x.decode("latin-1") if isinstance(x, bytes) else x for x in v.tolist()]
            else:
                val = v.item() if hasattr(v, "item") else v
            lay[name] = {"dtype": str(obj.dtype), "shape": list(obj.shape), "value": val}
    with h5py.File(path, "r") as f:
        f.visititems(visit)
    return lay


def state_of(km):
    s = km.kmer_sba_start_indices
    return {"min_kmer_len": int(km.min_kmer_len),
            "max_kmer_len": None if km.max_kmer_len is None else int(km.max_kmer_len),
            "kmer_source_strand": km.kmer_source_strand,
            "track_strands_separately": bool(km.track_strands_separately),
            "_is_initialized": bool(km._is_initialized), "_is_set": bool(km._is_set),
            "_is_sorted": bool(km._is_sorted),
            "kmer_sba_start_indices": None if s is None else [int(x) for x in s],
            "forward_sba": bytes(km.seq_coll.forward_sba).decode("latin-1"),
            "seg_starts": km.seq_coll._forward_sba_seg_starts.tolist(),
            "names": list(km.seq_coll.forward_record_names)}


def persistence_cases():
    out = []
    tmp = tempfile.mkdtemp(prefix="gk_persist_")
    for cname, seqs, mn, mx, sort in (("seq1_sorted", SEQ_LIST_1, 2, None, True),
                                       ("seq2_k3_sorted", SEQ_LIST_2, 3, 3, True),
                                       ("seq2_unsorted", SEQ_LIST_2, 1, 5, False)):
        sc = SequenceCollection(sequence_list=seqs, strands_to_load="forward")
        km = gk.Kmers(sc, min_kmer_len=mn, max_kmer_len=mx)
        if sort:
            km.kmer_sba_start_indices = mg.stable_sort(km)
            km._is_sorted = True
        h5 = os.path.join(HERE, f"persist_{cname}.h5")
        if os.path.exists(h5):
            os.remove(h5)
        km.save(h5, include_sequence_collection=True, format="hdf5")
        back = gk.Kmers()
        back.load(h5, format="hdf5")
        sh = os.path.join(tmp, cname)
        km.save(sh, include_sequence_collection=True, format="shelve")
        with shelve.open(sh) as db:
            keys = sorted(db.keys())
        back_sh = gk.Kmers()
        back_sh.load(sh, format="shelve")
        out.append({"name": cname, "h5_file": os.path.basename(h5), "h5_layout": h5_layout(h5),
                    "state_saved": state_of(km), "state_loaded_hdf5": state_of(back),
                    "state_loaded_shelve": state_of(back_sh), "shelve_keys": keys})
    return out


def main():
    doc = {"generator": "tests/golden/make_contracts.py", "reference": "mrperkett/genome-kmers v1.0.1",
           "kmers_init": kmers_init_cases(), "seqcoll_init": seqcoll_init_cases(), "fasta": fasta_cases(),
           "full_info": full_info_cases(), "persistence": persistence_cases()}
    with open(os.path.join(HERE, "contracts.json"), "w") as fh:
        json.dump(doc, fh, indent=1, default=lambda o: o.item() if hasattr(o, "item") else str(o))
    for k, v in doc.items():
        if isinstance(v, list):
            print(k, len(v))


if __name__ == "__main__":
    main()
