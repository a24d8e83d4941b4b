"""Test setup: import paths, the ``gpu`` marker, golden-vector loading.

``-m "not gpu"`` runs everywhere (oracle vs golden vectors, host-side API, ABI surface);
``-m gpu`` needs an MI355X and exercises libgkm.so through its C ABI.
"""

import json
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG_ROOT = ROOT / "genome-kmers_amd"
GOLDEN = ROOT / "tests" / "golden"
for p in (str(PKG_ROOT), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libgkm.so")


@pytest.fixture(autouse=True)
def _check_level_tile_totals(request, monkeypatch):
    """GPU tests: every MSD level re-reads its bucket scan and compares it with the tile / chunk
    totals the list counters carried (the product plans levels from those totals alone)."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    from genome_kmers import _native

    try:
        monkeypatch.setitem(_native.options, "GKM_TEST_CHECK_TILES", "1")
    except Exception:  # no library on this machine: the test itself reports that
        pass
    yield


def load_manifest():
    with open(GOLDEN / "manifest.json") as fh:
        return json.load(fh)["cases"]


def load_case(name):
    with np.load(GOLDEN / f"{name}.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def seq_list_of(case, arrays):
    """Rebuild the (name, seq) list of a golden case from its sba / seg_starts."""
    sba = arrays["sba"]
    starts = arrays["seg_starts"].astype(np.int64)
    ends = np.append(starts[1:] - 1, len(sba))
    return [(name, bytes(sba[b:e]).decode()) for name, b, e in zip(case["record_names"], starts, ends)]


@pytest.fixture(scope="session")
def manifest():
    return load_manifest()
