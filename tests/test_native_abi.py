"""CPU checks of the C ABI: the library loads (no GPU needed), exports every entry point
declared in include/recsys_amd.h with a ctypes signature, and rejects bad arguments before
launching anything."""
import ctypes
import os
import re

import pytest

import recsys_amd  # noqa: F401
from recsys_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "recsys_amd.h")


def _declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int64_t|int|const char\*)\s+(rsx_\w+)\(", text, flags=re.M)))


def test_header_declares_entry_points():
    names = _declared()
    assert "rsx_nce_grouped_fwd" in names and "rsx_seq_embed_fwd" in names
    assert len(names) >= 14


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    lib = _native.load()
    for name in _declared():
        assert hasattr(lib, name), f"{name} declared in recsys_amd.h but not exported"
        assert name in _native._SIGS, f"{name} has no ctypes signature in _native.py"
    assert lib.rsx_target_arch() == b"gfx950"


def test_library_is_built_from_this_tree():
    """rsx_build_hash() (csrc/Makefile's sha256 stamp of the sources) equals the hash of the sources
    in this tree: the .so the tests load is not a stale build."""
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    info = _native.build_info()
    assert info["fresh"], info


def _prototypes():
    """{name: parameter count} of every prototype in the header."""
    text = open(HEADER).read()
    out = {}
    for m in re.finditer(r"^(?:int64_t|int|const char\*)\s+(rsx_\w+)\(([^;]*?)\);", text, flags=re.M | re.S):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_ctypes_signatures_match_header_arity():
    protos = _prototypes()
    assert set(protos) == set(_declared())
    for name, n in protos.items():
        assert name in _native._SIGS, name
        assert len(_native._SIGS[name][1]) == n, f"{name}: header has {n} parameters, ctypes {len(_native._SIGS[name][1])}"


def test_argument_errors_are_reported_without_a_gpu():
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("library not built")
    lib = _native.load()
    # D = 100 is rejected before any launch
    rc = lib.rsx_gather_rows(None, 100, None, 10, 100, 0, 1e-12, None, None, None)
    assert rc == 1
    assert b"null tensor" in lib.rsx_last_error() or b"D must be" in lib.rsx_last_error()
    rc = lib.rsx_mha_fwd(ctypes.c_void_p(16), None, None, 2, 65, 4, 32, 1, 0.0, 0, ctypes.c_void_p(16), None, None)
    assert rc == 1 and b"L must be" in lib.rsx_last_error()
    rc = lib.rsx_nce_fwd(None, None, None, None, None, None, None, 4, 4, 128, 128, 0, 0.1, 3, 8, None, None, None)
    assert rc == 1 and b"unsupported flag" in lib.rsx_last_error()
    with pytest.raises(RuntimeError):
        _native.check(1, "probe")
