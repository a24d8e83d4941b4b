"""The reference-pinned host contracts of tests/test_contracts.py (SURVEY.md section 8 rows a1, a2,
f2, f4), repeated in the GPU tier: the driver's GPU run selects ``-m gpu`` only, and these checks
-- Kmers.__init__ errors, SequenceCollection construction, the native FASTA parser against the
reference loader's outputs, the shelve round trip -- must hold on the GPU box's build of libgkm
too.  Same fixtures, same assertions; HDF5 needs h5py, which the box lacks (container only)."""

import pytest

import test_contracts as tc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", [c for c in tc.KI if "error" in c["result"]],
                         ids=lambda c: f"{c['collection']}-{c['kwargs']}")
def test_kmers_init_errors_on_box(case):
    tc.test_kmers_init_errors(case)


@pytest.mark.parametrize("case", tc.C["seqcoll_init"], ids=lambda c: str(c["args"])[:60])
def test_seqcoll_init_on_box(case):
    tc.test_seqcoll_init(case)


@pytest.mark.parametrize("case", tc.C["fasta"], ids=lambda c: c["name"])
def test_fasta_matches_reference_loader_on_box(case, tmp_path):
    tc.test_fasta_matches_reference_loader(case, tmp_path)


@pytest.mark.parametrize("case", tc.PERSIST, ids=lambda c: c["name"])
def test_shelve_round_trip_matches_reference_on_box(case, tmp_path):
    tc.test_shelve_round_trip_matches_reference(case, tmp_path)
