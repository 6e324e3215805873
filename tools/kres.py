"""Per-kernel register / scratch / occupancy of a gfx950 build (hipcc's kernel-resource-usage
remarks), for checking that a change kept the hot kernels spill-free:

    python tools/kres.py [-D NAME=V ...] [--filter k_lml] [source.hip ...]

Compiles each translation unit (default: all of build.SOURCES) to a throw-away object under /tmp.
"""

from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from charon_amd import build  # noqa: E402

FIELDS = {"VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch", "Occupancy [waves/SIMD]": "occ",
          "LDS Size [bytes/block]": "lds", "SGPRs": "sgpr"}


def resources(srcs, defines=()):
    tmp = tempfile.mkdtemp(prefix="kres")
    procs = []
    for src in srcs:
        cmd = [build.HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", "--offload-device-only",
               "-Rpass-analysis=kernel-resource-usage"] + ["-D" + d for d in defines] + \
              [os.path.join(build.CSRC, src), "-o", os.path.join(tmp, src + ".o")]
        procs.append((src, subprocess.Popen(cmd, stderr=subprocess.PIPE, stdout=subprocess.DEVNULL, text=True)))
    out = {}
    for src, p in procs:
        err = p.communicate()[0 if False else 1]
        if p.returncode:
            raise RuntimeError(f"{src}: hipcc failed\n{err[-4000:]}")
        name = None
        for line in err.splitlines():
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                name = m.group(1)
                out[name] = {"src": src}
                continue
            for k, v in FIELDS.items():
                m = re.search(re.escape(k) + r": (\d+)", line)
                if m and name:
                    out[name][v] = int(m.group(1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sources", nargs="*")
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    res = resources(a.sources or build.SOURCES, a.D)
    for name, r in sorted(res.items(), key=lambda kv: (kv[1]["src"], kv[0])):
        if a.filter and a.filter not in name:
            continue
        if not name.startswith("_Z") or "k_" not in name:
            continue
        short = re.sub(r"^_ZN2hb\d+", "", name)
        print(f"{r['src']:15s} {short[:60]:60s} vgpr {r.get('vgpr', 0):4d} agpr {r.get('agpr', 0):3d} "
              f"scratch {r.get('scratch', 0):6d} occ {r.get('occ', 0)}")


if __name__ == "__main__":
    main()
