"""The C ABI library loads and exports every entry point include/gkm.h declares (CPU only)."""

import re

import pytest

from conftest import ROOT
from genome_kmers import _native


def header_symbols():
    text = (ROOT / "include" / "gkm.h").read_text()
    return sorted(set(re.findall(r"^(?:int|void|const char \*)\s*(gk_[a-z_]+)\s*\(", text, re.M)))


def test_library_built_and_loads():
    lib = _native.load_library()
    assert lib is not None


def test_exports_every_declared_symbol():
    lib = _native.load_library()
    declared = header_symbols()
    assert declared, "no declarations parsed"
    missing = [s for s in declared if not hasattr(lib, s)]
    assert missing == []
    assert sorted(_native.EXPORTED) == declared


def test_engine_fails_loudly_without_gpu():
    if _native.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_native.GkError, match="no CPU fallback"):
        _native.Engine()
