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
HEADERS = ["hd.h", "consts.h", "fp.h", "fr.h", "tower.h", "ec.h", "ec28.h", "sha256.h", "h2c.h", "pairing.h", "ops.h", "pair3.h",
           "pair6.h", "layout.h", "lines.h", "rlc.h", "ta_small.h", "pair28.h", "hostmul64.h", "coalesce.h", "msgtable.h"]


def _newer(target, deps):
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def build_id(defines=()) -> str:
    """The id embedded in the library: the source hash (charon_amd._lib.source_build_id) plus the
    tuning defines of a variant build."""
    from charon_amd._lib import BUILD_ID_PREFIX, source_build_id
    bid = BUILD_ID_PREFIX + source_build_id(ROOT)
    if defines:
        bid += "+" + ",".join(d.replace(" ", "") for d in defines)
    return bid


def build_library(force: bool = False, verbose: bool = True, defines=(), out: str = LIB) -> str:
    """defines / out: tuning variants (e.g. ("HB_OCC2=2",) -> charon_amd/lib/variants/...), used by
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


def build_hostcheck(force: bool = False, verbose: bool = True, defines=(), out: str = "") -> str:
    """defines / out: another build of the harness (e.g. ("HB_FP_ILP",): the two-accumulator
    products, tests/test_sanitizers.py)."""
    src = os.path.join(ROOT, "tests", "native", "hostcheck.cpp")
    out = out or os.path.join(ROOT, "tests", "native", "libhbls_hostcheck.so")
    deps = [src] + [os.path.join(CSRC, f) for f in HEADERS]
    if not force and _newer(out, deps):
        return out
    cmd = ["g++", "-O3", "-march=x86-64-v3", "-std=c++17", "-pthread", "-shared", "-fPIC", "-o", out + ".tmp", src]
    cmd[1:1] = ["-D" + d for d in defines]
    subprocess.run(cmd, check=True, timeout=900)
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"built {out}")
    return out


def build_hostcheck_sanitized(force: bool = False, verbose: bool = True) -> str:
    """The test harness under AddressSanitizer + UndefinedBehaviorSanitizer (host code only; the
    GPU build has no sanitizer here).  tests/test_sanitizers.py runs the host tests against it."""
    src = os.path.join(ROOT, "tests", "native", "hostcheck.cpp")
    out = os.path.join(ROOT, "tests", "native", "libhbls_hostcheck_asan.so")
    deps = [src] + [os.path.join(CSRC, f) for f in HEADERS]
    if not force and _newer(out, deps):
        return out
    cmd = ["g++", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-std=c++17", "-pthread", "-shared", "-fPIC", "-o", out + ".tmp", src]
    subprocess.run(cmd, check=True, timeout=900)
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"built {out}")
    return out


def main(argv=None):
    force = "--force" in (argv or sys.argv[1:])
    build_library(force)
    build_hostcheck(force)


if __name__ == "__main__":
    main()
