"""The host restatement of the kernels' arithmetic (tests/native/hostcheck.cpp, the same headers
the GPU kernels compile) under AddressSanitizer and UndefinedBehaviorSanitizer: the host-harness
tests run in a child process against the sanitized build (ASan runtime preloaded, leak detection
off -- the interpreter itself is not instrumented).  Any report aborts the child."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_harness_under_asan_ubsan():
    from charon_amd.build import build_hostcheck_sanitized
    try:
        lib = build_hostcheck_sanitized(verbose=False)
    except (subprocess.CalledProcessError, OSError) as e:  # no sanitizer runtime in this toolchain
        pytest.skip(f"sanitized build unavailable: {e}")
    asan = subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    env = dict(os.environ, HBLS_HOSTCHECK_LIB=lib, LD_PRELOAD=asan,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_hostcheck.py")],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=1500)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in tail and "runtime error" not in tail, tail

