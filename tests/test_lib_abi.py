"""CPU-side checks of the C-ABI library: it loads (no GPU needed) and exports
every symbol include/dlcs.h declares; no compute calls."""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "dlcs.h")
# a declaration: return type at the start of a line, then the dlcs_* name and "("
DECL = re.compile(r"^[A-Za-z_][A-Za-z0-9_ ]*[ *][ *]*(dlcs_[a-z0-9_]+)\s*\(", re.M)


def declared_symbols(diag=False):
    """dlcs_* functions declared in include/dlcs.h: the product library's, or (diag)
    those inside its DLCS_DIAG_BUILD blocks (libdlcs_hip_diag.so only)."""
    txt = open(HEADER).read()
    blocks = re.findall(r"#ifdef DLCS_DIAG_BUILD(.*?)#endif", txt, re.S)
    if diag:
        return sorted(set(DECL.findall("".join(blocks))))
    for b in blocks:
        txt = txt.replace(b, "")
    return sorted(set(DECL.findall(txt)))


def test_header_matches_binding():
    from dl_cs import _lib
    assert declared_symbols() == _lib.exported_symbols()
    assert declared_symbols(diag=True) == sorted(_lib.DIAG_SIGNATURES)


def test_library_exports_all_symbols():
    from dl_cs import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libdlcs_hip.so not built")
    L = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(L, name), name
    # the product library carries no DIAG-build entry point (one path per op)
    if os.path.basename(_lib.LIB_PATH) == "libdlcs_hip.so":
        for name in declared_symbols(diag=True):
            assert not hasattr(L, name), name
    L.dlcs_version.restype = ctypes.c_int
    assert L.dlcs_version() == 1
    L.dlcs_status_string.restype = ctypes.c_char_p
    assert L.dlcs_status_string(100001) == b"invalid argument"


def test_product_exports_equal_header():
    """The product library's dlcs_* export set is exactly the header's product section:
    nothing superseded or DIAG-only is reachable through the product ABI."""
    from dl_cs import _lib
    path = os.path.join(os.path.dirname(_lib.LIB_PATH), "libdlcs_hip.so")
    if not os.path.exists(path):
        pytest.skip("libdlcs_hip.so not built")
    nm = shutil.which("nm") or shutil.which("llvm-nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    if not os.path.exists(nm):
        pytest.skip("no nm to list the dynamic symbols")
    out = subprocess.run([nm, "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    exported = sorted({ln.split()[-1] for ln in out.splitlines() if ln.split() and ln.split()[-1].startswith("dlcs_")})
    assert exported == declared_symbols()
