"""Build provenance: libhipbls.so carries the hash of the sources it was built from
(hbls_build_id), charon_amd/build.py reuses a library only when that hash matches the tree, and the
loader refuses a library built from other sources (a stale .so next to edited kernels)."""
import os
import shutil

import pytest

from charon_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _copy_tree(tmp_path):
    shutil.copytree(os.path.join(ROOT, "charon_amd", "csrc"), tmp_path / "charon_amd" / "csrc")
    shutil.copytree(os.path.join(ROOT, "include"), tmp_path / "include")
    return str(tmp_path)


def test_source_id_tracks_every_header(tmp_path):
    root = _copy_tree(tmp_path)
    base = _lib.source_build_id(root)
    assert base == _lib.source_build_id(ROOT)
    hdr = tmp_path / "charon_amd" / "csrc" / "fp.h"
    hdr.write_text(hdr.read_text() + "\n// touched\n")
    assert _lib.source_build_id(root) != base
    (tmp_path / "include" / "hipbls.h").write_text("/* other */")
    assert len({base, _lib.source_build_id(root)}) == 2


def test_stale_library_is_refused(tmp_path):
    from charon_amd.build import build_library
    path = build_library(verbose=False)
    lib_id = _lib.embedded_build_id(path)
    assert lib_id.startswith(_lib.BUILD_ID_PREFIX)
    _lib.check_build_id(lib_id)  # the in-tree library matches the tree
    root = _copy_tree(tmp_path)
    hdr = tmp_path / "charon_amd" / "csrc" / "ec28.h"
    hdr.write_text(hdr.read_text() + "\n// touched\n")
    with pytest.raises(_lib.HipBlsUnavailable, match="stale"):
        _lib.check_build_id(lib_id, root)
    with pytest.raises(_lib.HipBlsUnavailable):
        _lib.check_build_id("hbls-build:unversioned")


def test_loaded_library_reports_its_id():
    from charon_amd.build import build_library, build_id
    L = _lib.load_library(build_library(verbose=False))
    assert L.hbls_build_id().decode() == build_id()
    # a variant build carries its defines after the hash; only the hash is compared
    _lib.check_build_id(build_id(("HB_X=1",)))


def _copy_harness_tree(tmp_path):
    root = _copy_tree(tmp_path)
    os.makedirs(tmp_path / "tests" / "native")
    shutil.copy(os.path.join(ROOT, "tests", "native", "hostcheck.cpp"), tmp_path / "tests" / "native")
    return root


def test_stale_cpu_harness_is_refused(tmp_path):
    """The g++ harness behind cpu_baseline and the host tests carries the hash of its sources and
    flags (hc_build_id); one built before a header changed is refused and rebuilt."""
    import ctypes
    from charon_amd import build
    path = build.build_hostcheck(verbose=False)
    hid = build.check_hostcheck(path)  # the in-tree harness matches the tree
    assert hid.startswith(build.HOSTCHECK_PREFIX)
    lib = ctypes.CDLL(path)
    lib.hc_build_id.restype = ctypes.c_char_p
    assert lib.hc_build_id().decode() == hid
    root = _copy_harness_tree(tmp_path)
    assert build.hostcheck_build_id(root=root) == hid
    hdr = tmp_path / "charon_amd" / "csrc" / "fp.h"
    hdr.write_text(hdr.read_text() + "\n// touched\n")
    with pytest.raises(RuntimeError, match="stale CPU harness"):
        build.check_hostcheck(path, root=root)
    # other flags or defines are another harness
    assert build.hostcheck_build_id(("HB_HOST_MUL28",)) != hid
    assert build.hostcheck_build_id(flags=build.SANITIZED_FLAGS) != hid
