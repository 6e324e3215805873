"""Build libhipbls.so (gfx950) in-tree, plus the test-only CPU harness.

    python -m charon_amd.build            # product library + test harness
The product library is compiled by hipcc for --offload-arch=gfx950 only.
"""

from __future__ import annotations

import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib", "libhipbls.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = ["hipbls.hip", "pipeline.hip", "threshold.hip", "vbatch.hip", "vgroup.hip", "roots.hip", "hash.hip", "msm.hip",
           "hashsplit.hip"]


def build_id(defines=()) -> str:
    """The id embedded in the library: the source hash (charon_amd._lib.source_build_id) plus the
    tuning defines of a variant build."""
    from charon_amd._lib import BUILD_ID_PREFIX, source_build_id
    bid = BUILD_ID_PREFIX + source_build_id(ROOT)
    if defines:
        bid += "+" + ",".join(d.replace(" ", "") for d in defines)
    return bid


def build_library(force: bool = False, verbose: bool = True, defines=(), out: str = LIB) -> str:
    """defines / out: experiment variants (-D defines -> charon_amd/lib/variants/...), used by
    tools/ experiments through HBLS_LIBRARY; the product is the default build.  A library whose
    embedded build id equals the tree's is reused; any other is rebuilt."""
    from charon_amd._lib import embedded_build_id
    LIB = out
    bid = build_id(defines)
    if not force and os.path.exists(LIB) and embedded_build_id(LIB) == bid:
        if verbose:
            print(f"reused {LIB} ({bid}: built from these sources)")
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    t = time.time()
    # the translation units compile in parallel (pipeline.hip is the long one), then link
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(os.path.dirname(LIB), os.path.splitext(src)[0] + ".o")
        objs.append(obj)
        extra = [f'-DHBLS_BUILD_ID="{bid}"'] if src == "hipbls.hip" else []
        procs.append(subprocess.Popen([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c"] +
                                      ["-D" + d for d in defines] + extra + [os.path.join(CSRC, src), "-o", obj]))
    for p in procs:
        if p.wait(timeout=3000) != 0:
            raise RuntimeError("hipcc failed")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB + ".tmp"] + objs +
                   ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"], check=True, timeout=600)
    os.replace(LIB + ".tmp", LIB)
    if verbose:
        print(f"compiled {LIB} in {time.time() - t:.1f}s ({bid})")
    return LIB


HOSTCHECK_PREFIX = "hbls-hostcheck:"
HOSTCHECK_FLAGS = ["-O3", "-march=x86-64-v3", "-std=c++17", "-pthread", "-shared", "-fPIC"]


def hostcheck_build_id(defines=(), flags=None, root: str = "") -> str:
    """The id embedded in the CPU harness: sha256 (16 hex digits) over the harness source, every
    header of charon_amd/csrc (it includes the kernels' arithmetic from there), the compiler flags
    and the defines -- what `hc_build_id()` of a harness built from this tree returns."""
    import hashlib
    root = root or ROOT
    csrc = os.path.join(root, "charon_amd", "csrc")
    h = hashlib.sha256()
    files = [os.path.join(root, "tests", "native", "hostcheck.cpp")] + \
        sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith(".h"))
    for f in files:
        h.update(os.path.relpath(f, root).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    h.update(" ".join((flags or HOSTCHECK_FLAGS) + ["-D" + d for d in defines]).encode())
    return HOSTCHECK_PREFIX + h.hexdigest()[:16]


def embedded_hostcheck_id(path: str) -> str:
    """The harness id inside a built harness file, read from its bytes (no loading)."""
    import re
    with open(path, "rb") as f:
        m = re.search(rb"hbls-hostcheck:[0-9a-f]{16}", f.read())
    return m.group(0).decode() if m else ""


def check_hostcheck(path: str, defines=(), root: str = "") -> str:
    """The harness's id if it was built from the tree's sources (with these defines), else raise:
    a stale harness would time or check code the kernels no longer run."""
    got, want = embedded_hostcheck_id(path), hostcheck_build_id(defines, root=root)
    if got != want:
        raise RuntimeError(f"stale CPU harness {path}: built as {got or '(unstamped)'}, the tree is {want}")
    return got


def build_hostcheck(force: bool = False, verbose: bool = True, defines=(), out: str = "") -> str:
    """defines / out: another build of the harness (e.g. ("HB_HOST_MUL28",): the 28-bit host
    products, tests/test_sanitizers.py).  A harness whose embedded id (hc_build_id) equals this
    tree's is reused; any other -- a header touched, other flags -- is rebuilt."""
    src = os.path.join(ROOT, "tests", "native", "hostcheck.cpp")
    out = out or os.path.join(ROOT, "tests", "native", "libhbls_hostcheck.so")
    bid = hostcheck_build_id(defines)
    if not force and os.path.exists(out) and embedded_hostcheck_id(out) == bid:
        return out
    cmd = ["g++"] + HOSTCHECK_FLAGS + ["-D" + d for d in defines] + [f'-DHC_BUILD_ID="{bid}"', "-o", out + ".tmp", src]
    subprocess.run(cmd, check=True, timeout=900)
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"built {out}")
    return out


def build_c_client(force: bool = False, verbose: bool = True) -> str:
    """tests/native/cabi_client: a C program linked against libhipbls.so through include/hipbls.h
    (what the Go shim's cgo does), compiled with -std=c99 -Wall -Wextra -Werror so the header is
    checked as C; test-only."""
    src = os.path.join(ROOT, "tests", "native", "cabi_client.c")
    out = os.path.join(ROOT, "tests", "native", "cabi_client")
    deps = [src, os.path.join(ROOT, "include", "hipbls.h")]
    if not force and os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps):
        return out
    cmd = ["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror", "-o", out + ".tmp", src,
           "-L" + os.path.dirname(LIB), "-lhipbls", "-Wl,-rpath," + os.path.dirname(LIB),
           "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, timeout=300)
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"built {out}")
    return out


SANITIZED_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                   "-fno-sanitize-recover=undefined", "-std=c++17", "-pthread", "-shared", "-fPIC"]


def build_hostcheck_sanitized(force: bool = False, verbose: bool = True) -> str:
    """The test harness under AddressSanitizer + UndefinedBehaviorSanitizer (host code only; the
    GPU build has no sanitizer here).  tests/test_sanitizers.py runs the host tests against it.
    Reused only when its embedded id matches the tree (as build_hostcheck)."""
    src = os.path.join(ROOT, "tests", "native", "hostcheck.cpp")
    out = os.path.join(ROOT, "tests", "native", "libhbls_hostcheck_asan.so")
    bid = hostcheck_build_id(flags=SANITIZED_FLAGS)
    if not force and os.path.exists(out) and embedded_hostcheck_id(out) == bid:
        return out
    cmd = ["g++"] + SANITIZED_FLAGS + [f'-DHC_BUILD_ID="{bid}"', "-o", out + ".tmp", src]
    subprocess.run(cmd, check=True, timeout=900)
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"built {out}")
    return out


def main(argv=None):
    force = "--force" in (argv or sys.argv[1:])
    build_library(force)
    build_hostcheck(force)
    build_c_client(force)


if __name__ == "__main__":
    main()
