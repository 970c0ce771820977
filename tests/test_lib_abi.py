"""CPU-side checks of the C-ABI library: it loads (no GPU needed) and exports
every symbol include/dlcs.h declares; no compute calls."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "dlcs.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(dlcs_[a-z0-9_]+)\s*\(", txt)))


def test_header_matches_binding():
    from dl_cs import _lib
    assert declared_symbols() == _lib.exported_symbols()


def test_library_exports_all_symbols():
    from dl_cs import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libdlcs_hip.so not built")
    L = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(L, name), name
    L.dlcs_version.restype = ctypes.c_int
    assert L.dlcs_version() == 1
    L.dlcs_status_string.restype = ctypes.c_char_p
    assert L.dlcs_status_string(100001) == b"invalid argument"
