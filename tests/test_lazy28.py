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


@pytest.mark.parametrize("field", ["Fp", "Fp2"])
def test_bounds(field):
    out = lazy28.check(lazy28.VMAX[field], (field,))
    assert all(v <= lazy28.VMAX[field] for v in out.values()), out


@pytest.mark.parametrize("field,prefix", [("Fp", "1"), ("Fp2", "2")])
def test_search_finds_no_smaller_constants(field, prefix):
    """the committed constants are the smallest the interval analysis admits at VMAX"""
    saved = dict(lazy28.KSITE)
    try:
        found = lazy28.search(lazy28.VMAX[field], (field,))
    finally:
        lazy28.KSITE.clear()
        lazy28.KSITE.update(saved)
    assert found == {k: v for k, v in saved.items() if k.startswith(prefix)}


def _fn(src, name):
    i = src.index(name + "(")
    return src[i:src.index("\n}\n", i)]


def test_constants_match_ec28():
    """each ec28.h formula uses exactly the constants lazy28.py proves for its sites"""
    src = open(os.path.join(ROOT, "charon_amd", "csrc", "ec28.h")).read()
    k = lazy28.KSITE

    def used(*names, pat=r"l_sub<(\d+), (\d+)>"):
        return sorted(tuple(map(int, m)) for n in names for m in re.findall(pat, _fn(src, n)))

    assert used("HDNI G1L g1l_dbl") == sorted([k["1D_D"], k["1D_X"], k["1D_W"], k["1D_Y"]])
    assert used("HD G1L g1l_add_tail") == sorted([k["1A_X"], k["1A_Y"], k["1A_W"]])
    assert used("HDNI G1L g1l_madd") == used("HDNI G1L g1l_add") == sorted([k["1A_H"], k["1A_R"]])
    assert used("HDNI G2L g2l_dbl", pat=r"f2l_sub<(\d+), (\d+)>") == sorted([k["2D_D"], k["2D_X"], k["2D_W"], k["2D_Y"]])
    assert used("HDNI G2L g2l_madd", pat=r"f2l_sub<(\d+), (\d+)>") == sorted(
        [k["2A_H"], k["2A_R"], k["2A_X"], k["2A_W"], k["2A_Y"]])
    assert used("HDNI G2L g2l_add", pat=r"f2l_sub<(\d+), (\d+)>") == sorted(
        [k["2J_H"], k["2J_R"], k["2J_X"], k["2J_W"], k["2J_Y"]])
    assert used("HD F2L f2l_sqr") == [k["2Q"]]
    # the G2 formulas square through the product policy (fs<S, T>) with the same constant
    assert set(used("HDNI G2L g2l_dbl", "HDNI G2L g2l_madd", "HDNI G2L g2l_add", pat=r"fs<(\d+), (\d+)>")) == {k["2Q"]}
    assert re.search(r"kF2N = k28_make\((\d+), (\d+)\)", src).groups() == tuple(map(str, k["2N"]))
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


def _random_twist_point(rng):
    while True:
        x = (rng.randrange(B.P), rng.randrange(B.P))
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B_G2))
        if y is not None:
            return (x, y)


def _check2(lib, pt):
    out = (ctypes.c_int * 3)()
    (x0, x1), (y0, y1) = pt
    raw = b"".join(v.to_bytes(48, "big") for v in (x0, x1, y0, y1))
    lib.hc_g2_subgroup2(raw, out)
    want = B.g2_in_subgroup(pt)
    assert out[0] == want and out[1] == want, (out[0], out[1], want)
    return out[2]


def test_g2_subgroup_lazy_matches(lib):
    """subgroup points, random twist points (not in G2) and the committed off-subgroup fixture"""
    import json
    lib.hc_g2_subgroup2.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
    rng = random.Random(282)
    pts = [B.G2_GEN, B.g2_neg(B.G2_GEN)] + [B.g2_mul(B.G2_GEN, rng.randrange(1, B.R)) for _ in range(3)]
    pts += [_random_twist_point(rng) for _ in range(6)]
    with open(os.path.join(ROOT, "tests", "golden", "off_subgroup_g2.json")) as f:
        for h in json.load(f)["points"][:4]:
            pts.append(B.g2_decompress(bytes.fromhex(h), subgroup_check=False))
    fpm = [_check2(lib, p) for p in pts]
    assert max(fpm) <= 1250  # 63 doublings x 17 + 5 mixed additions x 30 + psi / eq


def test_zero_test(lib):
    """l_is_zero (no product) agrees with the Montgomery-product form and with v % p on multiples
    of p up to 64 p, their neighbours, random values and lazy (uncarried) limb layouts"""
    lib.hc_l28_is_zero.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int)]
    rng = random.Random(2828)
    vals = []
    for k in range(65):
        for d in (0, 1, -1, 1 << 336, -(1 << 336), 1 << 200, rng.randrange(1, 1 << 300)):
            v = k * B.P + d
            if 0 <= v < (1 << 391):
                vals.append(v)
    vals += [rng.randrange(1 << 391) for _ in range(200)]
    for v in vals:
        limbs = lazy28.limbs28(v)
        layouts = [limbs]
        j = rng.randrange(13)  # the same value with a borrowed carry: limb j + 2^28, limb j+1 - 1
        if limbs[j + 1] > 0:
            l2 = list(limbs)
            l2[j] += 1 << 28
            l2[j + 1] -= 1
            layouts.append(l2)
        for lb in layouts:
            out = (ctypes.c_int * 2)()
            lib.hc_l28_is_zero((ctypes.c_uint32 * 14)(*lb), out)
            assert out[0] == out[1] == (v % B.P == 0), (v, lb, out[0], out[1])


def test_rlc_chunk_ladder_lazy(lib):
    """ec28.h g1l_msm_ladder (k_rlc_msm's G1 chunk ladder): sum [a_i + b_i lambda] P_i over chunks
    of 1, 2, 10 and 11 keys, including repeated keys and coefficients whose ladder meets +-T
    (equal keys, all-ones, single bits), against the oracle"""
    lib.hc_rlc_sum_g1_lazy.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p]
    lam = (-B.X_PARAM ** 2) % B.R
    rng = random.Random(2829)
    keys = [B.g1_mul(B.G1_GEN, rng.randrange(1, B.R)) for _ in range(6)]
    cases = []
    for k in (1, 2, 10, 11):
        pts = [keys[rng.randrange(len(keys))] for _ in range(k)]
        cases.append((pts, [(rng.getrandbits(32), rng.getrandbits(32)) for _ in range(k)]))
    cases.append(([keys[0]] * 4, [(1, 0), (1, 0), (0xFFFFFFFF, 0), (0, 1)]))   # R meets T: doubling
    cases.append(([keys[1], B.g1_neg(keys[1])], [(5, 0), (5, 0)]))             # sum is infinity
    cases.append(([keys[2]] * 3, [(0xFFFFFFFF, 0xFFFFFFFF)] * 3))
    for pts, ab in cases:
        buf = b"".join(B.g1_compress(p) for p in pts)
        flat = (ctypes.c_uint32 * (2 * len(ab)))(*[x for pair in ab for x in pair])
        out = ctypes.create_string_buffer(48)
        assert lib.hc_rlc_sum_g1_lazy(len(pts), buf, flat, out) == 0
        want = None
        for p, (a, b) in zip(pts, ab):
            want = B.g1_add(want, B.g1_mul(p, (a + b * lam) % B.R))
        assert out.raw == B.g1_compress(want)


def _sparse_digits(rng, k, cases):
    """k items' sparse-format records (ec28.h RLC_DIGITS) and their (A, B): random digits, plus
    the extreme strings (every digit (1, 1); every digit -(1, -1)) and an unusable item"""
    recs, ab = [], []
    for i in range(k):
        kind = cases[i % len(cases)]
        if kind == "rand":
            d = [rng.randrange(8) for _ in range(22)]
        elif kind == "max":
            d = [2] * 22
        else:  # "alt": -(1, -1) = (-1, 1)
            d = [7] * 22
        words = [0, 0, 0]
        for j, v in enumerate(d):
            words[j // 10] |= v << (3 * (j % 10))
        usable = kind != "skip"
        recs.append(words + [1 if usable else 0])
        A = B_ = 0
        for j, v in enumerate(d):
            u, w = [(1, 0), (0, 1), (1, 1), (1, -1)][v & 3]
            if v & 4:
                u, w = -u, -w
            A += u * 4 ** j
            B_ += w * 4 ** j
        ab.append((A, B_) if usable else (0, 0))
    return recs, ab


def test_rlc_sparse_chunk_ladders(lib):
    """ec28.h g1l/g2l_msm_ladder_sparse (k_rlc_msm's chunk ladders in the sparse coefficient
    format, the table built by rlc.h sparse_put / sparse_fix): sum [A_i + B_i lambda] P_i against
    the oracle, for chunks of 1, 7 and 16 items, repeated points (the ladder meets +-T), extreme
    digit strings and a skipped item; and the 8^22 digit strings are distinct coefficients (the
    base-4 {-1, 0, 1} digits are a unique representation: spot-checked on colliding neighbours)"""
    lam = (-B.X_PARAM ** 2) % B.R
    rng = random.Random(2833)
    for fn, argt in (("hc_rlc_sum_g1_sparse", 48), ("hc_rlc_sum_g2_sparse", 96)):
        getattr(lib, fn).argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p]
    g1 = [B.g1_mul(B.G1_GEN, rng.randrange(1, B.R)) for _ in range(5)]
    g2 = [B.g2_mul(B.G2_GEN, rng.randrange(1, B.R)) for _ in range(3)]
    plans = [(1, ["rand"]), (7, ["rand", "max", "rand", "skip", "alt"]), (16, ["rand"])]
    for k, kinds in plans:
        for side in (1, 2):
            pool = g1 if side == 1 else g2
            pts = [pool[rng.randrange(len(pool))] for _ in range(k)]
            if k == 7:
                pts[2] = pts[0]  # the same point twice
            recs, ab = _sparse_digits(rng, k, kinds)
            flat = (ctypes.c_uint32 * (4 * k))(*[x for r in recs for x in r])
            if side == 1:
                buf = b"".join(B.g1_compress(p) for p in pts)
                out = ctypes.create_string_buffer(48)
                assert lib.hc_rlc_sum_g1_sparse(k, buf, flat, out) == 0
                want = None
                for p, (a, b) in zip(pts, ab):
                    want = B.g1_add(want, B.g1_mul(p, (a + b * lam) % B.R))
                assert out.raw == B.g1_compress(want), (k, side)
            else:
                buf = b"".join(B.g2_compress(p) for p in pts)
                out = ctypes.create_string_buffer(96)
                assert lib.hc_rlc_sum_g2_sparse(k, buf, flat, out) == 0
                want = None
                for p, (a, b) in zip(pts, ab):
                    want = B.g2_add(want, B.g2_mul(p, (a + b * lam) % B.R))
                assert out.raw == B.g2_compress(want), (k, side)
    # uniqueness: strings differing in one digit give different (A, B); A + B lambda = A' + B'
    # lambda mod r with |A - A'|, |B - B'| < 2^45 forces equality (lambda's lattice has no
    # vector that short: a = b lambda mod r with 0 < |b| < 2^45 means |a| > 2^126)
    for _ in range(200):
        recs, ab = _sparse_digits(rng, 1, ["rand"])
        r0 = recs[0]
        j = rng.randrange(22)
        d = (r0[j // 10] >> (3 * (j % 10))) & 7
        r1 = list(r0)
        r1[j // 10] ^= ((d ^ ((d + 1 + rng.randrange(7)) % 8)) << (3 * (j % 10)))
        A0, B0 = ab[0]
        A1 = B1 = 0
        for jj in range(22):
            v = (r1[jj // 10] >> (3 * (jj % 10))) & 7
            u, w = [(1, 0), (0, 1), (1, 1), (1, -1)][v & 3]
            if v & 4:
                u, w = -u, -w
            A1 += u * 4 ** jj
            B1 += w * 4 ** jj
        assert (A0 + B0 * lam - A1 - B1 * lam) % B.R != 0


def test_g2_xabs_ladder_lazy(lib):
    """ec28.h g2l_mul_by_xabs_l (the hash's cofactor ladders, general Jacobian additions) against
    ec.h jac_mul_by_xabs and the oracle, on random twist points with random Z, subgroup points and
    infinity"""
    lib.hc_g2_mul_xabs2.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    rng = random.Random(2830)
    pts = [_random_twist_point(rng) for _ in range(4)] + [B.G2_GEN, B.g2_mul(B.G2_GEN, 12345)]
    for pt in pts + [None]:
        (x0, x1), (y0, y1) = pt if pt else ((0, 0), (1, 0))
        z = (rng.randrange(B.P), rng.randrange(B.P)) if pt else (0, 0)
        raw = b"".join(v.to_bytes(48, "big") for v in (x0, x1, y0, y1) + z)
        out = ctypes.create_string_buffer(192)
        assert lib.hc_g2_mul_xabs2(raw, out) == 0
        want = B.g2_compress(B.g2_mul(pt, -B.X_PARAM)) if pt else B.g2_compress(None)
        assert out.raw[:96] == want and out.raw[96:] == want


def test_rlc_chunk_ladder_g2_lazy(lib):
    """ec28.h g2l_msm_ladder (k_rlc_msm's per-group signature side) against the oracle, incl. equal
    points (the ladder meets T) and a sum at infinity"""
    lib.hc_rlc_sum_g2_lazy.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p]
    lam = (-B.X_PARAM ** 2) % B.R
    rng = random.Random(2831)
    pts_all = [B.g2_mul(B.G2_GEN, rng.randrange(1, B.R)) for _ in range(4)]
    cases = [([pts_all[rng.randrange(4)] for _ in range(7)], [(rng.getrandbits(32), rng.getrandbits(32)) for _ in range(7)]),
             ([pts_all[0]] * 3, [(1, 0), (1, 0), (0, 1)]),
             ([pts_all[1], B.g2_neg(pts_all[1])], [(9, 0), (9, 0)])]
    for pts, ab in cases:
        buf = b"".join(B.g2_compress(p) for p in pts)
        flat = (ctypes.c_uint32 * (2 * len(ab)))(*[x for pair in ab for x in pair])
        out = ctypes.create_string_buffer(96)
        assert lib.hc_rlc_sum_g2_lazy(len(pts), buf, flat, out) == 0
        want = None
        for p, (a, b) in zip(pts, ab):
            want = B.g2_add(want, B.g2_mul(p, (a + b * lam) % B.R))
        assert out.raw == B.g2_compress(want)


# ---- round 4: the Miller-loop arithmetic in lazy limbs (charon_amd/csrc/pair28.h)

def test_line_and_pair_bounds():
    """the chain's point and lines, and the three-lane Fp12 steps, stay reduced below 2p"""
    assert lazy28.check_lines(2) == {"dbl": 2.0, "add": 2.0}
    assert lazy28.check_pair() == {"sqr": 2.0, "line": 2.0}


FE_SITES = "CMFJ"  # the final exponentiation's sites among the "4" ones


@pytest.mark.parametrize("group,keep", [("lines", lambda k: k[0] == "3"),
                                        ("pair", lambda k: k[0] == "4" and k[1] not in FE_SITES),
                                        ("fe", lambda k: k[0] == "4" and k[1] in FE_SITES)])
def test_line_pair_constants_are_minimal(group, keep):
    saved = dict(lazy28.KSITE)
    try:
        found = lazy28.search(2, (group,))
    finally:
        lazy28.KSITE.clear()
        lazy28.KSITE.update(saved)
    if group == "fe":  # the squares' constant is the Miller loop's (larger than the FE alone needs)
        need = found.pop("4Q")
        assert need[0] <= saved["4Q"][0] and need[1] <= saved["4Q"][1]
    assert found == {k: v for k, v in saved.items() if keep(k)}


def test_fe_bounds():
    """the final exponentiation's lane operations keep the lane values reduced below 2p"""
    r = lazy28.check_fe()
    assert r["cyc"] == r["mul"] == r["conj"] == 2.0 and r["frob"] < 1.1


def test_constants_match_pair28():
    src = open(os.path.join(ROOT, "charon_amd", "csrc", "pair28.h")).read()
    k = lazy28.KSITE

    def used(name, pat):
        return sorted(tuple(map(int, m)) for m in re.findall(pat, _fn(src, name)))

    sub = r"f2l_sub<(\d+), (\d+)>"
    assert used("HD void l2_dbl_line", sub) == sorted([k["3D_a0"], k["3D_a1"], k["3D_AE"], k["3D_Y"]])
    assert used("HD void l2_dbl_line", r"f2l_xi<(\d+), (\d+)>") == [k["3D_xi"]]
    assert used("HD void l2_add_line", sub) == sorted(
        [k["3A_th"], k["3A_la"], k["3A_H"], k["3A_a0"], k["3A_a1"], k["3A_Y"], k["3A_GH"]])
    sq = {tuple(map(int, m)) for n in ("HD void l2_dbl_line", "HD void l2_add_line")
          for m in re.findall(r"fs<(\d+), (\d+)>", _fn(src, n))}
    assert sq == {k["3Q"]}
    # the Fp4 lane values: f4l_mul / f4l_sqr instantiations and the lane steps
    assert re.findall(r"f4l_sqr<(\d+), (\d+), (\d+), (\d+)>", _fn(src, "HD void g4_sqr_p1")) == [
        tuple(map(str, k["4Svxi"] + k["4Svy"]))] * 2
    assert k["4Swxi"] == k["4Svxi"] and k["4Swy"] == k["4Svy"]
    assert re.findall(r"f4l_sub<(\d+), (\d+)>", _fn(src, "HD F4L g4_sqr_p2")) == [tuple(map(str, k["4SD"]))]
    assert re.findall(r"f4l_mul_s<(\d+), (\d+)>", _fn(src, "HD F4L g4_sqr_p2")) == [tuple(map(str, k["4Ss"]))]
    assert re.findall(r"f4l_mul_s<(\d+), (\d+)>", _fn(src, "HD F4L g4_line_p2")) == [tuple(map(str, k["4Ls"]))]
    assert re.findall(r"f4l_mul<(\d+), (\d+), (\d+), (\d+)>", _fn(src, "HD F4L g4_line_p2")) == [
        tuple(map(str, k["4Lmxi"] + k["4Lmy"]))]
    assert re.findall(r"fs3<(\d+), (\d+)>", _fn(src, "HD F4L f4l_sqr")) == [tuple(map(str, k["4Q"]))]
    # the final exponentiation's lane operations
    assert k["4Cvxi"] + k["4Cvy"] == k["4Svxi"] + k["4Svy"]  # g4_cyc_p1 squares as g4_sqr_p1
    assert re.findall(r"f4l_sqr<(\d+), (\d+), (\d+), (\d+)>", _fn(src, "HD F4L g4_cyc_p1")) == [
        tuple(map(str, k["4Cvxi"] + k["4Cvy"]))]
    assert used("HD F4L g4_cyc_p2", r"f4l_mul_s<(\d+), (\d+)>") == [k["4Cs"]]
    assert used("HD F4L g4_cyc_p2", sub) == [k["4Cn"]] * 2
    assert re.findall(r"f4l_mul<(\d+), (\d+), (\d+), (\d+)>", _fn(src, "HD void g4_mul_p1")) == [
        tuple(map(str, k["4Mvxi"] + k["4Mvy"])), tuple(map(str, k["4Mwxi"] + k["4Mwy"]))]
    assert (k["4MD"], k["4Ms"]) == (k["4SD"], k["4Ss"])  # g4_mul recombines through g4_sqr_p2
    assert used("HD F4L g4_conj", sub) == [k["4Jn"]] * 2
    assert used("HD F4L g4_frob", r"l_sub<(\d+), (\d+)>") == [k["4Fn"]] * 2


def _f2(b):
    return (int.from_bytes(b[:48], "big"), int.from_bytes(b[48:96], "big"))


def test_line_chain28_matches(lib):
    """pair28.h line_chain28 (lazy limbs, lines reduced and joined) gives the stored-word chain's
    68 lines (lines.h line_chain), unevaluated and at -g1, below 2p, with the same product count, on
    subgroup points and random twist points.  Its doubling keeps T scaled by 4 (no halving: the same
    projective point), so line j comes out multiplied by a nonzero Fp2 factor c_j -- the same for its
    three coefficients, and killed by the final exponentiation (c_j^(p^2 - 1) = 1): checked as
    proportionality, and exact equality for the first line (T not yet scaled)."""
    lib.hc_line_chain28.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p,
                                    ctypes.POINTER(ctypes.c_ulonglong)]
    rng = random.Random(2840)
    pts = [B.G2_GEN, B.g2_mul(B.G2_GEN, rng.randrange(1, B.R))] + [_random_twist_point(rng) for _ in range(3)]
    for pt in pts:
        (x0, x1), (y0, y1) = pt
        raw = b"".join(v.to_bytes(48, "big") for v in (x0, x1, y0, y1))
        for ev in (0, 1):
            a = ctypes.create_string_buffer(68 * 288)
            b = ctypes.create_string_buffer(68 * 288)
            cnt = (ctypes.c_ulonglong * 2)()
            assert lib.hc_line_chain28(raw, ev, a, b, cnt) == 0, "a lazy line at or above 2p"
            assert a.raw[:288] == b.raw[:288]
            for j in range(68):
                s_ = [_f2(a.raw[288 * j + 96 * i:288 * j + 96 * i + 96]) for i in range(3)]
                l_ = [_f2(b.raw[288 * j + 96 * i:288 * j + 96 * i + 96]) for i in range(3)]
                k = next(i for i in range(3) if s_[i] != (0, 0))
                c = B.f2_mul(l_[k], B.f2_inv(s_[k]))  # the line's factor
                assert c != (0, 0) and all(B.f2_mul(c, s_[i]) == l_[i] for i in range(3)), j
            assert cnt[0] == cnt[1] == 1571 + (68 * 4 if ev else 0)


def test_lines_at_p_equal_evaluated_lines(lib):
    """pipeline.hip k_lines_at_p (the chain of H(m) evaluated at the group's P inside the chain, the
    distinct-message slots' path) gives exactly k_lines_msg + k_mml_eval's evaluated lines, every
    value below 2p, for G2 points and P on and off the generator's multiples (P = g1, random
    multiples, x = 0 edge coordinates)"""
    lib.hc_lines_at_p.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
    rng = random.Random(2842)
    qs = [B.G2_GEN, B.g2_mul(B.G2_GEN, rng.randrange(1, B.R)), _random_twist_point(rng)]
    ps = [B.G1_GEN, B.g1_mul(B.G1_GEN, rng.randrange(1, B.R)), B.g1_mul(B.G1_GEN, B.R - 1)]
    for q in qs:
        (x0, x1), (y0, y1) = q
        qraw = b"".join(v.to_bytes(48, "big") for v in (x0, x1, y0, y1))
        for p in ps:
            praw = p[0].to_bytes(48, "big") + p[1].to_bytes(48, "big")
            a = ctypes.create_string_buffer(68 * 288)
            b = ctypes.create_string_buffer(68 * 288)
            assert lib.hc_lines_at_p(qraw, praw, a, b) == 0, "a line at P at or above 2p"
            assert a.raw == b.raw


def _rand_f12(rng):
    return b"".join(rng.randrange(B.P).to_bytes(48, "big") for _ in range(12))


def test_g4_lane_ops_match_tower(lib):
    """the three-lane Fp12 square and sparse-line product of pair28.h (the roles run in turn with
    pair3.h's exchanges) equal tower.h's f12_sqr / f12_mul_line, on random values and edge values
    (zero, one, p - 1 coordinates)"""
    lib.hc_g4_ops.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
    rng = random.Random(2841)
    cases = [(_rand_f12(rng), b"".join(rng.randrange(B.P).to_bytes(48, "big") for _ in range(6))) for _ in range(8)]
    pm1 = (B.P - 1).to_bytes(48, "big")
    cases.append((pm1 * 12, pm1 * 6))
    cases.append(((1).to_bytes(48, "big") + bytes(48 * 11), bytes(48 * 6)))
    for f, ln in cases:
        out = ctypes.create_string_buffer(4 * 576)
        assert lib.hc_g4_ops(f, ln, out) == 0
        assert out.raw[0:576] == out.raw[576:1152], "g4_sqr"
        assert out.raw[1152:1728] == out.raw[1728:2304], "g4_mul_line"


def test_fe28_matches_tower(lib):
    """pair28.h's final exponentiation in lazy limbs (g4_cyc / g4_mul / g4_conj / g4_frob, the
    three roles run in turn with pair3.h's exchanges) equals pairing.h final_exponentiation, on
    random values and edge values (p - 1 coordinates, one)"""
    lib.hc_fe28.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    rng = random.Random(7741)
    cases = [_rand_f12(rng) for _ in range(3)]
    cases.append((B.P - 1).to_bytes(48, "big") * 12)
    cases.append((1).to_bytes(48, "big") + bytes(48 * 11))
    for f in cases:
        out = ctypes.create_string_buffer(2 * 576)
        assert lib.hc_fe28(f, out) == 0
        assert out.raw[:576] == out.raw[576:]
