"""Worst-case bound checker for the lazily reduced 28-bit-limb point arithmetic (csrc/ec28.h).

ec28.h keeps G1 / G2 Jacobian coordinates in 14 limbs of 28 bits between Montgomery products
and replaces the [0, 2p) additions/subtractions of fp.h with limb-wise ones: a + b, and
a + K - b with K a multiple of p whose limbs are spread so that every limb of K is at least the
matching limb of any admissible b (no borrows).  Nothing is carried until `norm` and nothing is
reduced modulo p outside the products, so every intermediate has a per-limb bound and a value
bound, and the formulas are only correct if
  * every limb stays below 2^32 (the limbs are 32-bit registers),
  * every column of a product -- sum of a_j b_(k-j) + sum m_j p_(k-j) + carry-in -- stays below
    2^64 (the one-register accumulators of fp.h), and the squaring's doubled limbs below 2^32,
  * every subtraction's K dominates the subtrahend limb by limb, and
  * every value stays below 2^392 (14 x 28 bits).
This module restates each ec28.h formula over intervals (`Bound`) and asserts those conditions
for the worst case of every input allowed by the loop invariant (the coordinates of a point
normalised, value < VMAX), then checks that the outputs satisfy the same invariant, so the
ladders can iterate.  tests/test_lazy28.py runs it; the host build of ec28.h is compared with
fp.h's arithmetic on concrete points there too.
"""

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
M28 = (1 << 28) - 1
R = 1 << 392
NLIMB = 14


def limbs28(v):
    return [(v >> (28 * i)) & M28 for i in range(NLIMB)]


P28 = limbs28(P)


def kconst(s, t):
    """Limbs of K = s p spread with redundancy t: K_0 = c_0 + t 2^28, K_i = c_i + t 2^28 - t
    (0 < i < 13), K_13 = c_13 - t; every low limb is >= t (2^28 - 1).  (ec28.h K28<s, t>)"""
    c = limbs28(P * s)
    assert (P * s) < (1 << 392)
    k = [c[0] + t * (1 << 28)] + [c[i] + t * (1 << 28) - t for i in range(1, 13)] + [c[13] - t]
    assert sum(x << (28 * i) for i, x in enumerate(k)) == P * s and k[13] >= 0
    return k


class Bound:
    """per-limb upper bounds and an upper bound of the value (all quantities are >= 0)"""

    def __init__(self, lb, v):
        self.lb = list(lb)
        self.v = v
        assert all(0 <= x < (1 << 32) for x in self.lb), self.lb
        assert v < R

    @staticmethod
    def normalised(vmax):
        return Bound([M28] * 13 + [vmax >> 364], vmax)


def add(a, b):
    return Bound([x + y for x, y in zip(a.lb, b.lb)], a.v + b.v)


def shl(a, s):
    return Bound([x << s for x in a.lb], a.v << s)


def sub(a, b, site):
    """a + K - b, K = kconst(*KSITE[site]) = s p"""
    s, t = KSITE[site]
    k = kconst(s, t)
    for i in range(NLIMB):
        assert k[i] >= b.lb[i], ("K does not dominate", site, s, t, i, k[i], b.lb[i])
    return Bound([x + y for x, y in zip(a.lb, k)], a.v + P * s)


def norm(a):
    # carry propagation: l[i+1] += l[i] >> 28 ; l[i] &= M28 -- the limbs never exceed 2^32 on the way
    carry = 0
    for i in range(13):
        x = a.lb[i] + carry
        assert x < (1 << 32)
        carry = x >> 28
    assert a.lb[13] + carry < (1 << 32)
    return Bound.normalised(a.v)


def _columns(a, b, square=False):
    if square:
        assert all(2 * x < (1 << 32) for x in a.lb)
    acc = 0
    for k in range(27):
        lo, hi = (0, k) if k < 14 else (k - 13, 13)
        s = sum(a.lb[j] * b.lb[k - j] for j in range(lo, hi + 1))
        s += sum(M28 * P28[k - j] for j in range(lo, hi + 1) if (j < k or k >= 14))
        if k < 14:
            s += M28 * P28[0]
        acc = s + (acc >> 28)
        assert acc < (1 << 64), ("column overflow", k, acc.bit_length(), max(a.lb).bit_length(), max(b.lb).bit_length())
    return acc


def mul(a, b):
    _columns(a, b)
    return Bound.normalised(a.v * b.v // R + P + 1)


def sqr(a):
    _columns(a, a, square=True)
    return Bound.normalised(a.v * a.v // R + P + 1)


# ---- Fp2 (u^2 = -1): real = a0 b0 + (K - a1) b1, imag = a0 b1 + a1 b0, one product-scanning pass
def f2(c0, c1):
    return (c0, c1)


def f2_add(a, b):
    return (add(a[0], b[0]), add(a[1], b[1]))


def f2_sub(a, b, site):
    return (sub(a[0], b[0], site), sub(a[1], b[1], site))


def f2_shl(a, s):
    return (shl(a[0], s), shl(a[1], s))


def f2_norm(a):
    return (norm(a[0]), norm(a[1]))


def f2_mul(a, b, site):
    """ec28.h f2l_mul: a1 enters the real column negated as K - a1"""
    na1 = sub(Bound([0] * NLIMB, 0), a[1], site)
    acc_r = acc_i = 0
    for k in range(27):
        lo, hi = (0, k) if k < 14 else (k - 13, 13)
        mp = sum(M28 * P28[k - j] for j in range(lo, hi + 1) if (j < k or k >= 14)) + (M28 * P28[0] if k < 14 else 0)
        sr = sum(a[0].lb[j] * b[0].lb[k - j] + na1.lb[j] * b[1].lb[k - j] for j in range(lo, hi + 1)) + mp
        si = sum(a[0].lb[j] * b[1].lb[k - j] + a[1].lb[j] * b[0].lb[k - j] for j in range(lo, hi + 1)) + mp
        acc_r = sr + (acc_r >> 28)
        acc_i = si + (acc_i >> 28)
        assert acc_r < (1 << 64) and acc_i < (1 << 64), ("Fp2 column overflow", k)
    vr = (a[0].v * b[0].v + na1.v * b[1].v) // R + P + 1
    vi = (a[0].v * b[1].v + a[1].v * b[0].v) // R + P + 1
    return (Bound.normalised(vr), Bound.normalised(vi))


def f2_sqr(a, site):
    """(a0 + a1)(a0 + K - a1) + 2 a0 a1 u: two Fp products"""
    return (mul(add(a[0], a[1]), sub(a[0], a[1], site)), mul(shl(a[0], 1), a[1]))


# ------------------------------------------------------------------------------------------
# The formulas of ec28.h, written over an abstract field (Fp: Bound, Fp2: pair) -- same order,
# same constants (the (s, t) pairs are the template arguments of the C++ code).
class FpOps:
    add = staticmethod(add)

    @staticmethod
    def sub(a, b, site):
        return sub(a, b, "1" + site)

    shl = staticmethod(shl)
    norm = staticmethod(norm)
    mul = staticmethod(mul)
    sqr = staticmethod(sqr)

    @staticmethod
    def nrm(vmax):
        return Bound.normalised(vmax)


class Fp2Ops:
    add = staticmethod(f2_add)

    @staticmethod
    def sub(a, b, site):
        return f2_sub(a, b, "2" + site)

    shl = staticmethod(f2_shl)
    norm = staticmethod(f2_norm)

    @staticmethod
    def mul(a, b):
        return f2_mul(a, b, "2N")

    @staticmethod
    def sqr(a):
        return f2_sqr(a, "2Q")

    @staticmethod
    def nrm(vmax):
        return (Bound.normalised(vmax), Bound.normalised(vmax))


# K = s p with redundancy t per subtraction site (ec28.h K28<s, t>; kept in sync by
# tests/test_lazy28.py, found by `python lazy28.py --search`)
VMAX = {"Fp": 20, "Fp2": 16}  # coordinates stay below VMAX p between the ladder steps
KSITE = {
    "1D_D": (3, 2), "1D_X": (17, 2), "1D_W": (19, 1), "1D_Y": (9, 8),
    "1A_H": (21, 1), "1A_R": (41, 2), "1A_X": (13, 12), "1A_W": (15, 1), "1A_Y": (9, 8),
    "2D_X": (9, 8), "2D_W": (11, 1), "2D_Y": (9, 8),
    "2A_H": (17, 1), "2A_R": (33, 2), "2A_X": (13, 12), "2A_W": (16, 1), "2A_Y": (9, 8),
    "2J_H": (2, 1), "2J_R": (3, 2), "2J_X": (13, 12), "2J_W": (15, 1), "2J_Y": (9, 8),
    "2N": (33, 6), "2Q": (36, 1),
}


def flat_bound(x):
    return x if isinstance(x, Bound) else None


def vmax_of(x):
    return x.v if isinstance(x, Bound) else max(x[0].v, x[1].v)


def dbl(F, X, Y, Z):
    """jac_dbl28 (dbl-2009-l)"""
    A = F.sqr(X)
    B = F.sqr(Y)
    C = F.sqr(B)
    T = F.sqr(F.add(X, B))
    E = F.add(F.add(A, A), A)
    Fv = F.sqr(E)
    D = F.norm(F.shl(F.sub(T, F.add(A, C), "D_D"), 1))
    X3 = F.norm(F.sub(Fv, F.shl(D, 1), "D_X"))
    W = F.sub(D, X3, "D_W")
    Y3 = F.norm(F.sub(F.mul(E, W), F.shl(C, 3), "D_Y"))
    Z3 = F.mul(F.shl(Y, 1), Z)
    return X3, Y3, Z3


def madd(F, X1, Y1, Z1, x2, y2):
    """jac_add_aff28 (madd-2007-bl with I = 4 HH folded into the shifts: J = 4 H HH, V = 4 X1 HH;
    Z3 = 2 Z1 H)"""
    Z1Z1 = F.sqr(Z1)
    U2 = F.mul(x2, Z1Z1)
    S2 = F.mul(F.mul(y2, Z1), Z1Z1)
    H = F.sub(U2, X1, "A_H")
    rr = F.norm(F.sub(F.shl(S2, 1), F.shl(Y1, 1), "A_R"))
    return _add_tail(F, H, rr, X1, Y1, F.shl(Z1, 1))


def _add_tail(F, H, rr, U1, S1, Zs):
    HH = F.sqr(H)
    J1 = F.mul(H, HH)                 # J = 4 J1
    V1 = F.mul(U1, HH)                # V = 4 V1
    X3 = F.norm(F.sub(F.sqr(rr), F.add(F.shl(J1, 2), F.shl(V1, 3)), "A_X"))
    Y3 = F.norm(F.sub(F.mul(rr, F.sub(F.shl(V1, 2), X3, "A_W")), F.shl(F.mul(S1, J1), 3), "A_Y"))
    Z3 = F.mul(Zs, H)
    return X3, Y3, Z3


def jadd(F, X1, Y1, Z1, X2, Y2, Z2):
    """jac_add28 (add-2007-bl with I = 4 HH as above; Z3 = 2 Z1 Z2 H)"""
    Z1Z1 = F.sqr(Z1)
    Z2Z2 = F.sqr(Z2)
    U1 = F.mul(X1, Z2Z2)
    U2 = F.mul(X2, Z1Z1)
    S1 = F.mul(F.mul(Y1, Z2), Z2Z2)
    S2 = F.mul(F.mul(Y2, Z1), Z1Z1)
    H = F.sub(U2, U1, "A_H")
    rr = F.norm(F.sub(F.shl(S2, 1), F.shl(S1, 1), "A_R"))
    return _add_tail(F, H, rr, U1, S1, F.mul(F.shl(Z1, 1), Z2))


def dbl2(F, X, Y, Z):
    """g2l_dbl: dbl-2009-l rearranged for the Fp2 products' bounds -- D = 4 X B from one product
    (the (X + B)^2 - A - C form grows D by its subtraction constant), E = 3A normalised before
    its square, E W = 3 (A W)"""
    A = F.sqr(X)
    B = F.sqr(Y)
    C = F.sqr(B)
    D1 = F.mul(X, B)                                  # D = 4 D1
    Fv = F.sqr(F.norm(F.add(F.shl(A, 1), A)))
    X3 = F.norm(F.sub(Fv, F.shl(D1, 3), "D_X"))
    W = F.sub(F.shl(D1, 2), X3, "D_W")
    AW = F.mul(W, A)
    Y3 = F.norm(F.sub(F.add(F.shl(AW, 1), AW), F.shl(C, 3), "D_Y"))
    Z3 = F.mul(F.shl(Y, 1), Z)
    return X3, Y3, Z3


def madd2(F, X1, Y1, Z1, x2, y2):
    """g2l_madd: madd-2007-bl as madd() with H normalised (its square is an Fp2 square)"""
    Z1Z1 = F.sqr(Z1)
    U2 = F.mul(x2, Z1Z1)
    S2 = F.mul(F.mul(y2, Z1), Z1Z1)
    H = F.norm(F.sub(U2, X1, "A_H"))
    rr = F.norm(F.sub(F.shl(S2, 1), F.shl(Y1, 1), "A_R"))
    HH = F.sqr(H)
    J1 = F.mul(H, HH)
    V1 = F.mul(X1, HH)
    X3 = F.norm(F.sub(F.sqr(rr), F.add(F.shl(J1, 2), F.shl(V1, 3)), "A_X"))
    Y3 = F.norm(F.sub(F.mul(F.sub(F.shl(V1, 2), X3, "A_W"), rr), F.shl(F.mul(Y1, J1), 3), "A_Y"))
    Z3 = F.mul(F.shl(Z1, 1), H)
    return X3, Y3, Z3


def jadd2(F, X1, Y1, Z1, X2, Y2, Z2):
    """g2l_add: add-2007-bl as jadd() with H normalised (its square is an Fp2 square)"""
    Z1Z1 = F.sqr(Z1)
    Z2Z2 = F.sqr(Z2)
    U1 = F.mul(X1, Z2Z2)
    U2 = F.mul(X2, Z1Z1)
    S1 = F.mul(F.mul(Y1, Z2), Z2Z2)
    S2 = F.mul(F.mul(Y2, Z1), Z1Z1)
    H = F.norm(F.sub(U2, U1, "J_H"))
    rr = F.norm(F.sub(F.shl(S2, 1), F.shl(S1, 1), "J_R"))
    HH = F.sqr(H)
    J1 = F.mul(H, HH)
    V1 = F.mul(U1, HH)
    X3 = F.norm(F.sub(F.sqr(rr), F.add(F.shl(J1, 2), F.shl(V1, 3)), "J_X"))
    Y3 = F.norm(F.sub(F.mul(F.sub(F.shl(V1, 2), X3, "J_W"), rr), F.shl(F.mul(S1, J1), 3), "J_Y"))
    Z3 = F.mul(F.mul(F.shl(Z1, 1), Z2), H)
    return X3, Y3, Z3


def fits(x, vmax):
    return vmax_of(x) <= vmax and all(
        all(l <= M28 for l in b.lb[:13]) and b.lb[13] <= (vmax >> 364) for b in ([x] if isinstance(x, Bound) else x))


def check(vmax, fields=("Fp", "Fp2")):
    """Fixed point: points with coordinates normalised and < vmax p stay so through dbl / madd /
    add, with the affine input of madd normalised and < 2p.  Returns the output bounds (units of p)."""
    out = {}
    for name, F in (("Fp", FpOps), ("Fp2", Fp2Ops)):
        if name not in fields:
            continue
        vm = vmax * P
        X = Y = Z = F.nrm(vm)
        aff = F.nrm(2 * P)
        ops = (("dbl", lambda: dbl(F, X, Y, Z)), ("madd", lambda: madd(F, X, Y, Z, aff, aff)),
               ("add", lambda: jadd(F, X, Y, Z, X, Y, Z)))
        if name == "Fp2":
            ops = (("dbl", lambda: dbl2(F, X, Y, Z)), ("madd", lambda: madd2(F, X, Y, Z, aff, aff)),
                   ("add", lambda: jadd2(F, X, Y, Z, X, Y, Z)))
        for op, fn in ops:
            res = fn()
            for c in res:
                assert fits(c, vm), (name, op, vmax_of(c) / P)
            out[(name, op)] = max(vmax_of(c) for c in res) / P
    return out


def search(vmax, fields=("Fp", "Fp2")):
    """smallest K per site (t from the subtrahend's limb bound, s from its value) for vmax"""
    global sub
    plain = sub
    need = {}

    def auto(a, b, site):
        t = max(1, -(-max(b.lb[:13]) // M28))
        s = 1
        while not all(k >= x for k, x in zip(kconst(s, t), b.lb)):
            s += 1
        old = need.get(site, (0, 0))
        need[site] = (max(old[0], s), max(old[1], t))
        KSITE[site] = need[site]
        return plain(a, b, site)

    sub = auto
    try:
        for _ in range(4):  # the sites feed each other: iterate to the fixed point
            check(vmax, fields)
    finally:
        sub = plain
    return dict(sorted(need.items()))


if __name__ == "__main__":
    import sys
    if "--search" in sys.argv:
        for vm in (16, 20, 24, 28, 32, 40, 48):
            try:
                ks = search(vm, tuple(a for a in ("Fp", "Fp2") if a in sys.argv) or ("Fp", "Fp2"))
                print(vm, ks)
            except AssertionError as e:
                print(vm, "fails:", e)
    else:
        for f in ("Fp", "Fp2"):
            for k, v in check(VMAX[f], (f,)).items():
                print(k, f"outputs < {v:.2f} p (VMAX {VMAX[f]})")
