"""C ABI: libdeapmi.so loads on a CPU-only host and exports every function
declared in include/deapmi.h (no compute calls without a GPU)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "deapmi.h")


def declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dm_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    names = declared()
    for must in ("dm_generation", "dm_evaluate", "dm_sel_tournament", "dm_sort_nondominated",
                 "dm_crowding_dist", "dm_sel_nsga2", "dm_mig_place", "dm_var_or"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from deap_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libdeapmi.so not built")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    # the Python binding binds the same set
    assert sorted(_lib.SIGNATURES) == declared()
    assert lib.dm_version  # callable without a GPU
    lib.dm_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.dm_version()


def test_struct_layouts_match_header():
    from deap_amd import _lib
    # dm_pop: 3 pointers + 2 int64 + 4 int32
    assert ctypes.sizeof(_lib.DevicePop) == 3 * 8 + 2 * 8 + 4 * 4
    assert ctypes.sizeof(_lib.Eval) == 8 + 8 + 8 * 8
    assert ctypes.sizeof(_lib.Variation) == 8 + 6 * 8 + 2 * 8
    assert ctypes.sizeof(_lib.Rng) == 16
    assert ctypes.sizeof(_lib.Decisions) == 9 * 8
    assert ctypes.sizeof(_lib.BoundedVar) == 2 * 4 + 6 * 8 + 2 * 8


def test_missing_library_fails_loudly(tmp_path):
    from deap_amd import _lib
    with pytest.raises(_lib.DeviceUnavailable):
        # a fresh loader pointed at a missing path must not fall back
        saved = _lib._lib
        _lib._lib = None
        try:
            _lib.load(str(tmp_path / "nope.so"))
        finally:
            _lib._lib = saved
