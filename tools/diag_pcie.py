"""Host-to-device copy rates at the host-buffer path's sizes (diagnosis for hipbls.hip's uploads):
pageable vs pinned source, one copy vs pieces, each timed with events on one stream.

    python tools/diag_pcie.py
"""
import json
import time

import numpy as np
import torch


def rate(src, dst, pieces=1, reps=5):
    s = torch.cuda.Stream()
    n = src.numel()
    step = (n + pieces - 1) // pieces
    best = 0.0
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            for o in range(0, n, step):
                dst[o:o + step].copy_(src[o:o + step], non_blocking=True)
        t1 = time.perf_counter()
        s.synchronize()
        t2 = time.perf_counter()
        best = max(best, n / (t2 - t0) / 1e9)
        enq = (t1 - t0) * 1e3
    return {"GB_per_s": round(best, 2), "enqueue_ms_last": round(enq, 3)}


def main():
    out = {}
    for mb in (67, 144):
        n = mb * 1000 * 1000
        dst = torch.empty(n, dtype=torch.uint8, device="cuda")
        page = torch.from_numpy(np.random.default_rng(1).integers(0, 256, n, dtype=np.uint8))
        pin = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        pin.copy_(page)
        t0 = time.perf_counter()
        pin.copy_(page)
        memcpy_ms = (time.perf_counter() - t0) * 1e3
        out[f"{mb}MB"] = {"pageable": rate(page, dst), "pinned": rate(pin, dst), "pinned_8_pieces": rate(pin, dst, 8),
                          "host_memcpy_to_pinned_ms": round(memcpy_ms, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
