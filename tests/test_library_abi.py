"""libhipbls.so loads on a CPU-only host and exports every entry point include/hipbls.h declares
(no compute calls: there is no GPU here)."""
import os
import re

from charon_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "hipbls.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hbls_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_all_symbols():
    from charon_amd.build import build_library
    L = _lib.load_library(build_library(verbose=False))
    for name in declared_symbols():
        assert hasattr(L, name), name


def test_library_is_gfx950_only():
    from charon_amd.build import build_library
    path = build_library(verbose=False)
    data = open(path, "rb").read()
    assert b"gfx950" in data
    assert b"gfx942" not in data and b"gfx90a" not in data
