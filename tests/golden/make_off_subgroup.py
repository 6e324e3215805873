"""Generate tests/golden/off_subgroup_g2.json: compressed G2 points on the curve but outside the
r-torsion subgroup (herumi's Sign.Deserialize rejects them: BAD_SIGNATURE), drawn with a fixed seed
by the oracle (test infrastructure).  bench.py's adversarial workload (C5) reads them as data.

    python tests/golden/make_off_subgroup.py
"""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import bls12381 as B  # noqa: E402


def main(count=16, seed=20251017):
    rng = random.Random(seed)
    out = []
    while len(out) < count:
        x = (rng.randrange(B.P), rng.randrange(B.P))
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B_G2))
        if y is None or B.g2_in_subgroup((x, y)):
            continue
        out.append(B.g2_compress((x, y)).hex())
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "off_subgroup_g2.json")
    with open(path, "w") as f:
        json.dump({"seed": seed, "points": out}, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
