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


def test_options_are_explicit_overrides():
    """gk_set_option: GKM_* test/tuning overrides set and cleared through _native.options; other
    names are refused (no compute call: runs without a GPU)."""
    lib = _native.load_library()
    assert lib.gk_set_option(b"NOT_A_KNOB", b"1") == _native.GK_E_ARG
    _native.options["GKM_TEST_PAIRS"] = "1"
    assert _native.options.get("GKM_TEST_PAIRS") == "1"
    del _native.options["GKM_TEST_PAIRS"]
    assert "GKM_TEST_PAIRS" not in _native.options
    assert lib.gk_set_option(b"GKM_TEST_PAIRS", None) == _native.GK_OK  # clearing an unset one is fine
