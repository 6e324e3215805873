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
    "2D_D": (3, 2), "2D_X": (5, 2), "2D_W": (7, 1), "2D_Y": (9, 8),
    "2A_H": (17, 1), "2A_R": (33, 2), "2A_X": (13, 12), "2A_W": (16, 1), "2A_Y": (9, 8),
    "2J_H": (2, 1), "2J_R": (3, 2), "2J_X": (13, 12), "2J_W": (15, 1), "2J_Y": (9, 8),
    "2N": (33, 6), "2Q": (36, 1),
    # round 4 (pair28.h): the Miller chain ("3") and the three-lane Fp4 values ("4"), proven at 2p
    "3A_GH": (6, 1), "3A_H": (3, 2), "3A_Y": (2, 1), "3A_a0": (2, 1), "3A_a1": (5, 1), "3A_la": (2, 1),
    "3A_th": (2, 1), "3D_AE": (113, 3), "3D_Y": (47, 12), "3D_a0": (38, 1), "3D_a1": (4, 3), "3D_xi": (2, 1),
    "3Q": (78, 1),
    "4Lmxi": (2, 1), "4Lmy": (3, 2), "4Ls": (2, 1), "4Q": (9, 2), "4SD": (9, 2), "4Ss": (14, 4),
    "4Svxi": (2, 1), "4Svy": (3, 2), "4Swxi": (2, 1), "4Swy": (3, 2),
    # the final exponentiation's lane operations (cyclotomic square "C", product "M", conjugate "J",
    # Frobenius "F"); they share 4Q with the Miller loop's squares
    "4Cn": (5, 2), "4Cs": (5, 1), "4Cvxi": (2, 1), "4Cvy": (3, 2), "4Fn": (3, 1), "4Jn": (3, 1),
    "4MD": (9, 2), "4Ms": (14, 4), "4Mvxi": (2, 1), "4Mvy": (3, 2), "4Mwxi": (2, 1), "4Mwy": (3, 2),
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
    """g2l_dbl: dbl-2009-l (2M + 5S) with D = 2((X + B)^2 - A - C) partially reduced (red, no
    product): unreduced, D's subtraction constant grows the point past VMAX; X + B and E = 3A
    normalised before their squares"""
    A = F.sqr(X)
    B = F.sqr(Y)
    C = F.sqr(B)
    T = F.sqr(F.norm(F.add(X, B)))
    E = F.norm(F.add(F.shl(A, 1), A))
    Fv = F.sqr(E)
    D = f2_red(F.shl(F.sub(T, F.add(A, C), "D_D"), 1))
    X3 = F.norm(F.sub(Fv, F.shl(D, 1), "D_X"))
    W = F.sub(D, X3, "D_W")
    Y3 = F.norm(F.sub(F.mul(W, E), F.shl(C, 3), "D_Y"))  # W first: 33p - W.c1 (2N) dominates
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


# ------------------------------------------------------------------------------------------
# Round 4: the Miller-loop arithmetic in lazy limbs (csrc/pair28.h).
#
# red(a): the partial reduction l_red of pair28.h -- a normalised value v < 2^390 becomes v - q p
# with q = floor(v / p) or one less, read off the top 56 bits (no product): normalised, < 2p.
def red(a):
    assert a.v < (1 << 390)  # the limbs need no carry pass (Bound keeps them below 2^32)
    return Bound.normalised(2 * P)


def f2_red(a):
    return (red(a[0]), red(a[1]))


def bmax(a, b):
    """the bound of a value that is a or b (the lane roles' selects of pair28.h)"""
    if isinstance(a, Bound):
        return Bound([max(x, y) for x, y in zip(a.lb, b.lb)], max(a.v, b.v))
    return tuple(bmax(x, y) for x, y in zip(a, b))


class LineOps(Fp2Ops):
    """the Fp2 of the line chain and the Fp4 lane arithmetic: its own squaring constant"""

    @staticmethod
    def sqr(a):
        return f2_sqr(a, "3Q")

    @staticmethod
    def sub(a, b, site):
        return f2_sub(a, b, "3" + site)


def f2_xi(F, a, site):
    """(a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u"""
    return (sub(a[0], a[1], "3" + site), add(a[0], a[1]))


ZERO2 = (Bound([0] * NLIMB, 0), Bound([0] * NLIMB, 0))


def ldbl(F, X, Y, Z):
    """pair28.h l2_dbl_line: the doubling step of the Miller chain in homogeneous projective
    coordinates on the twist (b' = 4 xi), scaled by 4 so that no halving is needed:
      A = Y^2, B = Z^2, C = 3 b' B = 12 xi B, E = 3 C, D = Y Z
      line (a0, a1, b1) = (A - C, -3 X^2, 2 D)
      X3 = 2 X Y (A - E), Y3 = (A + E)^2 - 12 C^2, Z3 = 8 A D
    The point's coordinates are reduced (l_red) at the end of every step: they stay below 2p."""
    A = F.sqr(Y)
    B = F.sqr(Z)
    xb = F.norm(f2_xi(F, B, "D_xi"))
    C = F.norm(F.add(F.shl(xb, 3), F.shl(xb, 2)))
    E = F.add(F.shl(C, 1), C)
    D = F.mul(Y, Z)
    XX = F.sqr(X)
    a0 = F.sub(A, C, "D_a0")
    a1 = F.sub(ZERO2, F.add(F.shl(XX, 1), XX), "D_a1")
    b1 = F.shl(D, 1)
    XY = F.mul(F.shl(X, 1), Y)
    X3 = f2_red(F.mul(XY, F.norm(F.sub(A, E, "D_AE"))))
    C2 = F.sqr(C)
    Y3 = f2_red(F.sub(F.sqr(F.norm(F.add(A, E))), F.add(F.shl(C2, 3), F.shl(C2, 2)), "D_Y"))
    Z3 = f2_red(F.shl(F.mul(A, D), 3))
    return (X3, Y3, Z3), (f2_red(a0), f2_red(a1), f2_red(b1))


def ladd(F, X, Y, Z, xq, yq):
    """pair28.h l2_add_line: T + Q for an affine Q, the chord through T and Q:
      th = Y - yq Z, la = X - xq Z, C = th^2, D = la^2, E = la D, F = Z C, G = X D,
      H = E + F - 2G; line (th xq - la yq, -th, la); X3 = la H, Y3 = th (G - H) - Y E, Z3 = Z E"""
    th = F.norm(F.sub(Y, F.mul(yq, Z), "A_th"))
    la = F.norm(F.sub(X, F.mul(xq, Z), "A_la"))
    C = F.sqr(th)
    D = F.sqr(la)
    E = F.mul(la, D)
    Fv = F.mul(Z, C)
    G = F.mul(X, D)
    H = F.norm(F.sub(F.add(E, Fv), F.shl(G, 1), "A_H"))
    a0 = F.sub(F.mul(th, xq), F.mul(la, yq), "A_a0")
    a1 = F.sub(ZERO2, th, "A_a1")
    X3 = f2_red(F.mul(la, H))
    Y3 = f2_red(F.sub(F.mul(th, F.norm(F.sub(G, H, "A_GH"))), F.mul(Y, E), "A_Y"))
    Z3 = f2_red(F.mul(Z, E))
    return (X3, Y3, Z3), (f2_red(a0), f2_red(a1), f2_red(la))


# Fp4 = Fp2[s]/(s^2 - xi) as (x, y); the lane values of pair28.h's three-lane Fp12
def f4_add(a, b):
    return (f2_add(a[0], b[0]), f2_add(a[1], b[1]))


def f4_sub(a, b, site):
    return (f2_sub(a[0], b[0], "4" + site), f2_sub(a[1], b[1], "4" + site))


def f4_norm(a):
    return (f2_norm(a[0]), f2_norm(a[1]))


def f4_red(a):
    return (f2_red(a[0]), f2_red(a[1]))


def f4_xi(a, site):
    return (sub(a[0], a[1], "4" + site), add(a[0], a[1]))


def f4_mul(a, b, site):
    """g4 Karatsuba: t0 = a.x b.x, t1 = a.y b.y, t2 = (a.x + a.y)(b.x + b.y);
    (t0 + xi t1, t2 - t0 - t1), normalised"""
    t0 = f2_mul(a[0], b[0], "2N")
    t1 = f2_mul(a[1], b[1], "2N")
    t2 = f2_mul(f2_add(a[0], a[1]), f2_add(b[0], b[1]), "2N")
    return f4_norm((f2_add(t0, f4_xi(t1, site + "xi")), f2_sub(t2, f2_add(t0, t1), "4" + site + "y")))


def f4_sqr(a, site):
    """(x + y s)^2 = (x^2 + xi y^2, (x + y)^2 - x^2 - y^2), normalised"""
    t0 = f2_sqr(a[0], "4Q")
    t1 = f2_sqr(a[1], "4Q")
    return f4_norm((f2_add(f4_xi(t1, site + "xi"), t0),
                    f2_sub(f2_sqr(f2_norm(f2_add(a[0], a[1])), "4Q"), f2_add(t0, t1), "4" + site + "y")))


def f4_mul_s(a, site):
    return (f4_xi(a[1], site), a[0])


def g4_sqr(A):
    """pair28.h g4_sqr (pair3.h g_sqr): sa = A_p + A_q, v = A^2, w = sa^2, D = w - v_p - v_q,
    C = Y + [k != 2] s X with (X, Y) = (D, v_e) or (v_e, D); reduced"""
    sa = f4_add(A, A)
    v = f4_sqr(A, "Sv")
    w = f4_sqr(sa, "Sw")
    D = f4_sub(w, f4_add(v, v), "SD")
    X = bmax(D, v)
    Y = bmax(v, D)
    sx = bmax(f4_mul_s(X, "Ss"), X)
    return f4_red(f4_add(Y, sx))


def g4_mul_line(Fv, a0, a1, b1):
    """pair28.h g4_mul_line (pair3.h g_mul_line): F (a0 + b1 s) + [s] F_n a1; reduced"""
    Qn = (f2_mul(Fv[0], a1, "2N"), f2_mul(Fv[1], a1, "2N"))
    Qs = bmax(f4_mul_s(Qn, "Ls"), Qn)
    return f4_red(f4_add(f4_mul(Fv, (a0, b1), "Lm"), Qs))


def check_lines(vmax):
    """the chain's point stays normalised below vmax p; the lines come out reduced (< 2p)"""
    F = LineOps
    vm = vmax * P
    X = Y = Z = F.nrm(vm)
    q = F.nrm(2 * P)
    out = {}
    for op, fn in (("dbl", lambda: ldbl(F, X, Y, Z)), ("add", lambda: ladd(F, X, Y, Z, q, q))):
        pt, line = fn()
        for c in pt:
            assert fits(c, vm), ("lines", op, vmax_of(c) / P)
        for c in line:
            assert fits(c, 2 * P)
        out[op] = max(vmax_of(c) for c in pt) / P
    return out


def check_pair():
    """the three-lane Fp12 value: lane values normalised below 2p (reduced after every step), the
    lines' coefficients below 2p"""
    A = (Fp2Ops.nrm(2 * P), Fp2Ops.nrm(2 * P))
    ln = Fp2Ops.nrm(2 * P)
    out = {}
    for op, fn in (("sqr", lambda: g4_sqr(A)), ("line", lambda: g4_mul_line(A, ln, ln, ln))):
        r = fn()
        assert all(fits(c, 2 * P) for c in r), op
        out[op] = max(vmax_of(c) for c in r) / P
    return out


# the final exponentiation's lane operations (pair28.h g4_cyc / g4_mul / g4_conj / g4_frob)
def g4_cyc(A):
    """pair28.h g4_cyc_p1 / g4_cyc_p2 (pair3.h g_cyclo_sqr): t = A^2 (sent to role e(k)); from the
    received te: ts = s te for k = 1, else te; (3 ts.x - 2 A.x, 3 ts.y + 2 A.y), for k = 1
    (3 ts.x + 2 A.x, 3 ts.y - 2 A.y), the negated terms as K - 2A; reduced"""
    t = f4_sqr(A, "Cv")
    ts = bmax(f4_mul_s(t, "Cs"), t)
    x3 = f2_add(f2_shl(ts[0], 1), ts[0])
    y3 = f2_add(f2_shl(ts[1], 1), ts[1])
    ax2, ay2 = f2_shl(A[0], 1), f2_shl(A[1], 1)
    nx, ny = f2_sub(ZERO2, ax2, "4Cn"), f2_sub(ZERO2, ay2, "4Cn")
    return f4_red((f2_add(x3, bmax(ax2, nx)), f2_add(y3, bmax(ay2, ny))))


def g4_mul(A, B):
    """pair28.h g4_mul_p1 / g4_mul_p2 (pair3.h g_mul): v = A B, w = (A_p + A_q)(B_p + B_q) with the
    sums normalised, the recombination of g4_sqr with its own constants; reduced"""
    v = f4_mul(A, B, "Mv")
    w = f4_mul(f4_norm(f4_add(A, A)), f4_norm(f4_add(B, B)), "Mw")
    D = f4_sub(w, f4_add(v, v), "MD")
    X = bmax(D, v)
    Y = bmax(v, D)
    sx = bmax(f4_mul_s(X, "Ms"), X)
    return f4_red(f4_add(Y, sx))


def g4_conj(A):
    """pair28.h g4_conj: (K - x, y) for k = 1, else (x, K - y); reduced"""
    return f4_red((bmax(A[0], f2_sub(ZERO2, A[0], "4Jn")), bmax(A[1], f2_sub(ZERO2, A[1], "4Jn"))))


def g4_frob(A, c):
    """pair28.h g4_frob: the Fp2 coefficients conjugated (odd J: c1 -> K - c1), times the reduced
    constants -- products of reduced values, below 2p without a reduction"""
    def cj(a):
        return (a[0], bmax(a[1], sub(ZERO2[0], a[1], "4Fn")))
    return (f2_mul(cj(A[0]), c, "2N"), f2_mul(cj(A[1]), c, "2N"))


def check_fe():
    """the final exponentiation's lane values: reduced (< 2p) in, reduced out, every operation"""
    A = (Fp2Ops.nrm(2 * P), Fp2Ops.nrm(2 * P))
    c = Fp2Ops.nrm(2 * P)
    out = {}
    for op, fn in (("cyc", lambda: g4_cyc(A)), ("mul", lambda: g4_mul(A, A)), ("conj", lambda: g4_conj(A)),
                   ("frob", lambda: g4_frob(A, c))):
        r = fn()
        assert all(fits(x, 2 * P) for x in r), op
        out[op] = max(vmax_of(x) for x in r) / P
    return out


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
        if site == "2N" and ("lines" in fields or "pair" in fields or "fe" in fields):
            return plain(a, b, site)  # the f2l_mul leaf's constant is shared: fixed
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
            if "lines" in fields:
                check_lines(vmax)
            elif "pair" in fields:
                check_pair()
            elif "fe" in fields:
                check_fe()
            else:
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
