"""The lazily reduced 28-bit-limb ladders (charon_amd/csrc/ec28.h).

* charon_amd/tools/lazy28.py restates every ec28.h formula over per-limb intervals: no limb
  leaves 32 bits, no product column 64 bits, every subtraction constant K = s p dominates its
  subtrahend limb by limb, and a point's coordinates return below VMAX p, so the ladders iterate;
* the constants K28<s, t> in ec28.h are the ones the checker proves;
* the host build of ec28.h (tests/native/hostcheck.cpp) decides G1 membership exactly as the
  stored-word ec.h test and the oracle do, on subgroup points, random curve points and points
  with a component in each prime-order subgroup of the cofactor (3, 11, 10177, 859267, 52437899).
"""
import ctypes
import os
import random
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "charon_amd", "tools"))
import lazy28  # noqa: E402
from oracle import bls12381 as B  # noqa: E402


def test_bounds_fp():
    out = lazy28.check(lazy28.VMAX, ("Fp",))
    assert all(v <= lazy28.VMAX for v in out.values()), out


def test_search_finds_no_smaller_constants():
    """the committed constants are the smallest the interval analysis admits at VMAX"""
    found = lazy28.search(lazy28.VMAX, ("Fp",))
    assert found == {k: v for k, v in lazy28.KSITE.items() if k.startswith("1")}


def test_constants_match_ec28():
    src = open(os.path.join(ROOT, "charon_amd", "csrc", "ec28.h")).read()
    used = {tuple(map(int, m)) for m in re.findall(r"l_sub<(\d+), (\d+)>", src)}
    want = {v for k, v in lazy28.KSITE.items() if k.startswith("1")}
    assert used == want, (used, want)
    kp = [int(x, 16) for x in re.search(r"kP28_\[14\] = \{([^}]*)\}", src).group(1).replace("u", "").split(",")]
    assert kp == lazy28.P28


@pytest.fixture(scope="module")
def lib():
    from charon_amd.build import build_hostcheck
    lb = ctypes.CDLL(os.environ.get("HBLS_HOSTCHECK_LIB") or build_hostcheck(verbose=False))
    lb.hc_g1_subgroup2.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
    return lb


def _random_curve_point(rng):
    while True:
        x = rng.randrange(B.P)
        y = B.fp_sqrt((x * x * x + 4) % B.P)
        if y is not None:
            return (x, y if rng.random() < 0.5 else (B.P - y) % B.P)


def _check(lib, pt):
    out = (ctypes.c_int * 3)()
    lib.hc_g1_subgroup2(pt[0].to_bytes(48, "big") + pt[1].to_bytes(48, "big"), out)
    want = B.g1_in_subgroup(pt)
    assert out[0] == want and out[1] == want, (pt, out[0], out[1], want)
    return out[2]


def test_g1_subgroup_lazy_matches(lib):
    rng = random.Random(28)
    n = B.H1 * B.R  # #E(Fp)
    pts = [B.G1_GEN, B.g1_neg(B.G1_GEN), B.g1_mul(B.G1_GEN, 2), B.g1_mul(B.G1_GEN, B.R - 1)]
    pts += [B.g1_mul(B.G1_GEN, rng.randrange(1, B.R)) for _ in range(4)]
    pts += [_random_curve_point(rng) for _ in range(6)]
    for ell in (3, 11, 10177, 859267, 52437899):
        v = 0
        while B.H1 % ell ** (v + 1) == 0:
            v += 1
        assert v >= 1
        for _ in range(2):
            t = None
            while t is None:  # a point of the ell-part of E(Fp) (order dividing ell^v; O: retry)
                t = B.g1_mul(_random_curve_point(rng), n // ell ** v)
            pts += [t, B.g1_add(t, B.g1_mul(B.G1_GEN, rng.randrange(1, B.R)))]
    fpm = [_check(lib, p) for p in pts]
    assert max(fpm) <= 1040  # two 63-step ladders: 126 doublings x 7 + 5 x 11 + 5 x 16 + phi/eq 8
