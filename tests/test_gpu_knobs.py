"""Every tuning setting of the library at a non-default value (no switch
without a test that runs it), -m gpu.

* In-process: the chunking of large verifications (hbls_tune HBLS_GROUP_CHUNK, HBLS_FALLBACK_CHUNK,
  HBLS_GROUP_MAX) at small values, so one call runs several pairing chunks and fallback passes --
  every status, and the first-error index, equal to the default run's.
* A child process per environment set (tests/gpu_helpers/env_child.py): every variable hbls_init
  reads, each at a non-default value, then Verify / first-error Verify / ThresholdAggregate /
  concurrent single-item callers checked against the construction.  The other setters
  (hbls_fe_batch, hbls_slot_msm, hbls_rlc_lanes, hbls_ta_joint, hbls_single_max, hbls_adaptive,
  hbls_sig_cache, hbls_dec_pair_max and the latency layouts of hbls_tune) have their own tests in
  tests/test_gpu_scale.py, tests/test_gpu_parity.py and tests/test_gpu_sigcache.py.
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from charon_amd import _lib
from charon_amd._lib import OK

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _p(x):
    return ctypes.c_void_p(x.ctypes.data)


@pytest.fixture(scope="module")
def L(hipbls):
    return _lib.load_library()


def _tune(L, name, value):
    prev = ctypes.c_size_t(0)
    assert L.hbls_tune(name.encode(), value, ctypes.byref(prev)) == 0, L.hbls_last_error()
    return prev.value


def test_chunked_verification_equals_default(L):
    import bench
    wl = dict(validators=12_000, n=7, t=5, distinct=False, n_msgs=64)
    d = dict(bench.setup_inputs(L, wl, wl["validators"], 0))
    d["sigs"] = d["sigs"].copy()
    bench.corrupt(L, d, 0.01, seed=31)
    NP = d["NP"]

    def both():
        st = np.full(NP, 255, dtype=np.uint8)
        assert L.hbls_verify_batch(_p(d["pks"]), _p(d["sigs"]), _p(d["item_msgs"]), _p(d["item_off"]),
                                   _p(d["item_len"]), NP, _p(st)) == 0, L.hbls_last_error()
        first = ctypes.c_int64(-2)
        fst = ctypes.c_uint8(0)
        assert L.hbls_verify_batch_first_error(_p(d["pks"]), _p(d["sigs"]), _p(d["item_msgs"]), _p(d["item_off"]),
                                               _p(d["item_len"]), NP, ctypes.byref(first), ctypes.byref(fst),
                                               None) == 0, L.hbls_last_error()
        return st, first.value, fst.value

    base = both()
    assert np.array_equal(base[0], d["exp_v"])
    assert base[1] == int(np.nonzero(d["exp_v"] != OK)[0][0])
    for name, value in (("HBLS_GROUP_CHUNK", 1000), ("HBLS_FALLBACK_CHUNK", 97), ("HBLS_GROUP_MAX", 3)):
        prev = _tune(L, name, value)
        try:
            st, f, fs = both()
        finally:
            _tune(L, name, prev)
        assert np.array_equal(st, base[0]), name
        assert (f, fs) == base[1:], name
    # all three at once
    prevs = [_tune(L, n, v) for n, v in (("HBLS_GROUP_CHUNK", 777), ("HBLS_FALLBACK_CHUNK", 50), ("HBLS_GROUP_MAX", 5))]
    try:
        st, f, fs = both()
    finally:
        for n, p in zip(("HBLS_GROUP_CHUNK", "HBLS_FALLBACK_CHUNK", "HBLS_GROUP_MAX"), prevs):
            _tune(L, n, p)
    assert np.array_equal(st, base[0]) and (f, fs) == base[1:]


# every variable hbls_init reads (charon_amd/csrc/hipbls.hip init_mask, coalesce_params), each at a
# value other than its default; two sets, since some pairs exclude each other's paths
ENV_SETS = [
    {"HBLS_DEVICE_MASK": "1", "HBLS_WS_SETS": "1", "HBLS_COALESCE_US": "0", "HBLS_COALESCE_MAX": "4",
     "HBLS_COALESCE_INFLIGHT": "1", "HBLS_HOST_TIMING": "1", "HBLS_STATS": "1", "HBLS_SIG_CACHE": "0",
     "HBLS_ADAPTIVE": "0", "HBLS_FE_BATCH": "0", "HBLS_SLOT_MSM": "0", "HBLS_SINGLE_MAX": "0",
     "HBLS_GROUP_CHUNK": "64", "HBLS_FALLBACK_CHUNK": "16", "HBLS_GROUP_MAX": "2", "HBLS_RLC_LANES": "1",
     "HBLS_TA_JOINT": "1", "HBLS_DEC_PAIR_MAX": "100000", "HBLS_TA_PAIR_MAX": "0", "HBLS_HASH_PAIR_MAX": "0",
     "HBLS_HASH_ONE_LANE": "0", "HBLS_HASH_SPLIT": "0", "HBLS_FE18_MAX": "0"},
    {"HBLS_WS_SETS": "5", "HBLS_COALESCE_US": "2000", "HBLS_COALESCE_MAX": "3", "HBLS_COALESCE_INFLIGHT": "2",
     "HBLS_SIG_CACHE": "1024", "HBLS_FE_BATCH": "4", "HBLS_SLOT_MSM": "64", "HBLS_SINGLE_MAX": "1",
     "HBLS_RLC_LANES": "128", "HBLS_TA_JOINT": "3", "HBLS_TA_PAIR_MAX": "100000", "HBLS_HASH_PAIR_MAX": "100000",
     "HBLS_HASH_ONE_LANE": "100000", "HBLS_FE18_MAX": "100000", "HBLS_GROUP_MAX": "64"},
    # one host-call context: every call reuses the staging buffers the previous call's
    # signature-cache put reads (the race fixed by hc_ready)
    {"HBLS_WS_SETS": "1", "HBLS_SIG_CACHE": "4096"},
]


@pytest.mark.parametrize("env", ENV_SETS, ids=["set0", "set1", "one_context"])
def test_environment_settings(env):
    child_env = {k: v for k, v in os.environ.items() if not k.startswith("HBLS_")}
    child_env.update(env)
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "gpu_helpers", "env_child.py")],
                       env=child_env, capture_output=True, text=True, timeout=240)
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert p.returncode == 0 and lines, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    res = json.loads(lines[-1])
    assert res["env"] == env
    assert all(res[k] for k in ("verify_ok", "first_error_ok", "aggregate_ok", "back_to_back_ok",
                                "single_callers_ok")), res
    if env.get("HBLS_HOST_TIMING") == "1":
        assert "hbls " in p.stderr  # the host-timing lines
