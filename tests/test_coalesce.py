"""The coalescing queue of concurrent single-item Verify callers (charon_amd/csrc/coalesce.h, used
by hbls_verify_batch) on the CPU with a stub batch runner: every request completes exactly once with
its own statuses, at most HBLS_COALESCE_INFLIGHT batches run at once, and requests arriving while a
batch runs lead a second batch instead of waiting behind it."""
import ctypes

import pytest


@pytest.fixture(scope="module")
def hc():
    from charon_amd.build import build_hostcheck
    lib = ctypes.CDLL(build_hostcheck(verbose=False))
    lib.hc_coalesce_stress.argtypes = [ctypes.c_int] * 5 + [ctypes.POINTER(ctypes.c_int)]
    return lib


def _stress(hc, threads, reqs, inflight, window_us, run_us):
    out = (ctypes.c_int * 5)()
    assert hc.hc_coalesce_stress(threads, reqs, inflight, window_us, run_us, out) == 0
    return {"max_running": out[0], "batches": out[1], "wrong_runs": out[2], "bad_status": out[3],
            "max_active": out[4]}


@pytest.mark.parametrize("inflight", [1, 2, 3])
def test_every_request_once_and_inflight_bound(hc, inflight):
    r = _stress(hc, threads=24, reqs=40, inflight=inflight, window_us=200, run_us=400)
    assert r["wrong_runs"] == 0 and r["bad_status"] == 0, r
    assert r["max_running"] <= inflight and r["max_active"] <= inflight, r
    assert r["batches"] < 24 * 40  # requests were coalesced


def test_late_arrivals_lead_a_second_batch(hc):
    """with batches much longer than the gathering window, callers arriving while one runs form and
    start the next: two (or three) batches overlap"""
    r = _stress(hc, threads=16, reqs=20, inflight=3, window_us=100, run_us=3000)
    assert r["wrong_runs"] == 0 and r["bad_status"] == 0, r
    assert r["max_running"] >= 2, r


def test_no_coalescing_window(hc):
    """window 0: every leader runs what is queued at once; still exactly once each"""
    r = _stress(hc, threads=8, reqs=25, inflight=2, window_us=0, run_us=50)
    assert r["wrong_runs"] == 0 and r["bad_status"] == 0 and r["max_running"] <= 2, r
