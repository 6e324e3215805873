"""The slot-wide check's bucket method (charon_amd/csrc/msm.hip) restated over the integers: the
scalar digits, the counting sort into buckets, the running-sum weighing of chunks of MSM_CHUNK buckets
plus one (lo - 1) multiple, the window shift and the final sum must give sum_i r_i x_i exactly.
Group elements are replaced by integers (the method only adds, doubles and scales), so this pins
the index arithmetic of k_msm_count / k_msm_fill / k_msm_order / k_msm_bucket / k_msm_reduce /
k_msm_sum without a GPU."""
import random

from charon_amd import opcounts

C, W, CHUNK = opcounts.MSM_C, opcounts.MSM_WINDOWS, opcounts.MSM_CHUNK
KEYS = W << C
MASK = (1 << C) - 1


def msm_int(points, coefs):
    """points[i] = (x, y): the two 'points' of item i (sig, -psi^2 sig); coefs[i] = (a, b)."""
    cnt = [0] * KEYS
    for a, b in coefs:
        for s in (a, b):
            for w in range(W):
                d = (s >> (C * w)) & MASK
                if d:
                    cnt[(w << C) + d] += 1
    off = [0] * (KEYS + 1)
    for k in range(KEYS):
        off[k + 1] = off[k] + cnt[k]
    cur = [0] * KEYS
    ent = [None] * off[KEYS]
    for i, (a, b) in enumerate(coefs):
        for h, s in enumerate((a, b)):
            for w in range(W):
                d = (s >> (C * w)) & MASK
                if d:
                    k = (w << C) + d
                    ent[off[k] + cur[k]] = (i << 1) | h
                    cur[k] += 1
    order = sorted(range(KEYS), key=lambda k: -min(cnt[k], 255))  # k_msm_order: any order sums the same
    bucket = [0] * KEYS
    for k in order:
        bucket[k] = sum(points[u >> 1][u & 1] for u in ent[off[k]:off[k + 1]])
    parts = []
    per_w = (1 << C) // CHUNK
    for c in range(KEYS // CHUNK):
        w, lo = c // per_w, (c % per_w) * CHUNK
        B = bucket[(w << C) + lo:(w << C) + lo + CHUNK]
        R = T = 0
        for j in range(CHUNK - 1, -1, -1):
            R += B[j]
            T += R
        Wc = T - R if lo == 0 else T + (lo - 1) * R
        parts.append(Wc << (C * w))
    return sum(parts)


def test_bucket_method_matches_direct_sum():
    rng = random.Random(11)
    n = 3000
    points = [(rng.randrange(1 << 40), rng.randrange(1 << 40)) for _ in range(n)]
    coefs = [(rng.randrange(1 << 32), rng.randrange(1 << 32)) for _ in range(n)]
    coefs[5] = (0, 0)           # an item outside the combination
    coefs[6] = (1, 0)           # coefficient one (a folded aggregate without batching)
    coefs[7] = (0xFFFFFFFF, 0xFFFF0000)
    direct = sum(a * x + b * y for (x, y), (a, b) in zip(points, coefs))
    assert msm_int(points, coefs) == direct
