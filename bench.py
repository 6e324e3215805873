#!/usr/bin/env python3
"""bench.py -- charon's BLS hot path on MI355X (BASELINE.json metric).

One step = one attestation slot of BASELINE.json configs[2] ("C3", the largest single-GPU
config): for V = 100 000 validators of a 10-operator threshold-7 cluster, each attesting to its
own AttestationData,
  0. build the slot's 100 000 signing roots from the SSZ AttestationData on device
     (eth2util/signing/signing.go:63-77 GetDataRoot; charon_amd/csrc/roots.hip)
  1. hash them to G2 (+ their Miller lines)
  2. verify all V*n = 1 000 000 partial signatures            (tbls.Verify,
     /root/reference/tbls/herumi.go:288-304; callers core/parsigex/parsigex.go:93-98)
  3. threshold-aggregate every validator's first t = 7 partials  (tbls.ThresholdAggregate,
     herumi.go:249-286; caller core/sigagg/sigagg.go:105)
  4. verify every aggregate under the validator's DV public key (core/sigagg/sigagg.go:117).
Steps 1-4 are one hbls_slot_device call (include/hipbls.h).  Inputs (compressed pubshares, partial
signatures, DV public keys, AttestationData, share indices) are resident in HBM before the timed
region; outputs are per-item status bytes and 96-byte aggregates in HBM.  Three consecutive slots
are in flight (--inflight), each on its own stream with its own outputs.

value = (verified partials + threshold aggregates) per second summed over all ranks; the
post-aggregate verifications are extra work not counted in it.  Weak scaling: every rank owns
its own V validators (validator sharding); with N > 1 ranks each step ends with the
library's RCCL all-gather of verdicts and aggregates over xGMI (hbls_allgather_device).

roofline: integer VALU: the dominant kernel's algorithmic Fp products (textbook
count, charon_amd/opcounts.py) x 300 multiply-adds, over its HIP-event time in the timed region,
against the measured v_mad_u64_u32 peak.
cpu_baseline: the same per-item arithmetic compiled for the host by g++ (tests/native/hostcheck.cpp,
a port -- herumi and the Go toolchain are absent), timed on a bounded sample of validators.
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import threading
import time

import numpy as np

# One hardware queue per stream: three slots in flight x (the slot's stream + its workspace set's
# four side streams) + the library stream.  With HIP's default of four, streams share queues and a
# latency-bound kernel (one final exponentiation, a hashing stage of 64 messages) holds up
# whatever else sits in its queue: C3 106.4 -> 101.3 ms, C2 16.7 -> 16.0 ms per slot on one box
# (profiles/r03j_*) with 16; 32 (the most the pool allows) adds C2 +2.6 %, C3 and C5 unchanged
# (profiles/r04q32_hw_queues_ab.txt).  Set before anything initialises the HIP runtime, over the environment's
# value (the GPU pool exports HIP's default of four); HBLS_HW_QUEUES chooses another count (at most
# 32).  A charon process sets it the same way in its environment.
os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(1, int(os.environ.get("HBLS_HW_QUEUES", "32")))))

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from charon_amd import opcounts  # noqa: E402

METRIC = "verified partial sigs/sec + ThresholdAggregate/sec per node, 1-8 MI355X"

WORKLOADS = {
    "c3": dict(validators=100_000, n=10, t=7, distinct=True, n_msgs=0,
               desc="C3 (BASELINE configs[2]): 100k validators, 10-operator threshold-7 cluster, distinct "
                    "per-validator messages: 1M partial Verify + 100k ThresholdAggregate (+100k aggregate Verify)"),
    "c2": dict(validators=10_000, n=4, t=3, distinct=False, n_msgs=64,
               desc="C2 (BASELINE configs[1]): 10k validators, 4-operator threshold-3 cluster, one attestation "
                    "slot with 64 committee signing roots: 40k partial Verify + 10k ThresholdAggregate "
                    "(+10k aggregate Verify)"),
    "c5": dict(validators=125_000, n=7, t=5, distinct=False, n_msgs=64, adversarial=0.01,
               desc="C5 (BASELINE configs[4]) per-GPU shard: the C4 shard with 1% of the partials corrupted in "
                    "equal fifths (random bytes, off-subgroup points, wrong message, another share's partial, "
                    "infinity), verdicts checked bit-exact against construction; sync-committee "
                    "VerifyAggregate over 512 keys per message timed beside it"),
    "c4": dict(validators=125_000, n=7, t=5, distinct=False, n_msgs=64,
               desc="C4 (BASELINE configs[3]) per-GPU shard: 1M validators over 8 GPUs = 125k validators, "
                    "7-operator threshold-5 cluster, 64 committee signing roots: 875k partial Verify + 125k "
                    "ThresholdAggregate (+125k aggregate Verify) per GPU"),
}


def _p(x) -> ctypes.c_void_p:
    """Device pointer of a torch tensor or host pointer of a numpy array."""
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        return ctypes.c_void_p(x.ctypes.data)
    return ctypes.c_void_p(x.data_ptr())


def _chk(L, rc):
    if rc != 0:
        raise RuntimeError("hipbls: " + L.hbls_last_error().decode(errors="replace"))


def attestation_data(roots, rank):
    """One synthetic phase0.AttestationData per message, SSZ-encoded (128 B): slot, committee
    index, beacon block root (the cluster's synthetic root), source and target checkpoints."""
    out = np.zeros((len(roots), 128), dtype=np.uint8)
    slot = 9_000_000 + rank
    for i, r in enumerate(roots):
        b = (slot.to_bytes(8, "little") + (i % 64).to_bytes(8, "little") + r +
             (slot // 32 - 1).to_bytes(8, "little") + r[::-1] + (slot // 32).to_bytes(8, "little") + r[16:] + r[:16])
        out[i] = np.frombuffer(b, dtype=np.uint8)
    return out.reshape(-1)


def attester_domain():
    """compute_domain(DOMAIN_BEACON_ATTESTER, fork version, genesis validators root)
    (eth2util/signing/signing.go:37-61 via the beacon node's Domain endpoint)."""
    import hashlib
    fork, gvr = bytes.fromhex("05000000"), hashlib.sha256(b"synthetic genesis").digest()
    fork_data_root = hashlib.sha256(fork + bytes(28) + gvr).digest()
    return np.frombuffer(bytes.fromhex("01000000") + fork_data_root[:28], dtype=np.uint8).copy()


def ta_share_positions(n, t):
    """The share positions (0-based) of the aggregated partials: a fixed pseudo-random t-subset of
    the n operators whose Lagrange coefficients at 0 are not all integers (runs of consecutive
    indices give integer coefficients, binomials, which shorten the aggregation ladders)."""
    import itertools
    import random
    from fractions import Fraction
    rng = random.Random(1000 * n + t)
    subsets = list(itertools.combinations(range(n), t))
    rng.shuffle(subsets)
    for pos in subsets:
        ids = [p + 1 for p in pos]
        lam = [Fraction(1)] * t
        for a, i in enumerate(ids):
            for j in ids:
                if j != i:
                    lam[a] *= Fraction(j, j - i)
        if any(x.denominator != 1 for x in lam):
            return list(pos)
    return list(range(t))


def corrupt(L, d, frac, seed, classes=(0, 1, 2, 3, 4)):
    """C5: corrupt `frac` of the partials in equal fifths (core/parsigex/parsigex_test.go:285-289,
    core/sigagg/sigagg_test.go:46-67 classes) and derive every expected status by construction:
      0 random 96 bytes without the compression flag   -> BAD_SIGNATURE (undecodable)
      1 an on-curve point outside G2 (tests/golden/off_subgroup_g2.json) -> BAD_SIGNATURE
      2 the partial signed over another message        -> NOT_VERIFIED
      3 another share's valid partial of the validator -> NOT_VERIFIED
      4 the infinity encoding                          -> NOT_VERIFIED
    The aggregation sees the corrupted signatures of its members: an undecodable member makes the
    validator's ThresholdAggregate BAD_SIGNATURE, any other corrupted member a wrong aggregate whose
    post-aggregate verification fails (NOT_VERIFIED)."""
    import hashlib
    import json
    import random
    n, t, V, NP = d["n"], d["t"], d["V"], d["NP"]
    rng = random.Random(seed)
    bad = rng.sample(range(NP), int(NP * frac))
    cls = {i: k % 5 for k, i in enumerate(bad) if k % 5 in classes}  # (classes: a subset, diagnosis)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden", "off_subgroup_g2.json")) as f:
        offsub = [bytes.fromhex(x) for x in json.load(f)["points"]]
    sigs = d["sigs"].reshape(NP, 96)
    orig = sigs.copy()
    exp_v = np.zeros(NP, dtype=np.uint8)
    wm = [i for i, c in cls.items() if c == 2]
    if wm:
        other = hashlib.sha256(b"another signing root").digest()
        msgs = np.frombuffer(other * len(wm), dtype=np.uint8).copy()
        sks = np.concatenate([d["sks"][32 * i:32 * i + 32] for i in wm])
        out = np.zeros(96 * len(wm), dtype=np.uint8)
        st = np.zeros(len(wm), dtype=np.uint8)
        off = np.arange(len(wm), dtype=np.uint64) * 32
        ln = np.full(len(wm), 32, dtype=np.uint32)
        _chk(L, L.hbls_sign_batch(_p(sks), _p(msgs), _p(off), _p(ln), len(wm), _p(out), _p(st)))
        assert not st.any()
        sigs[wm] = out.reshape(-1, 96)
    for i, c in cls.items():
        v, sh = divmod(i, n)
        if c == 0:
            b = bytearray(rng.randrange(256) for _ in range(96))
            b[0] &= 0x7F
            sigs[i] = np.frombuffer(bytes(b), dtype=np.uint8)
            exp_v[i] = 2
        elif c == 1:
            sigs[i] = np.frombuffer(offsub[i % len(offsub)], dtype=np.uint8)
            exp_v[i] = 2
        elif c == 2:
            exp_v[i] = 3
        elif c == 3:
            sigs[i] = orig[v * n + (sh + 1) % n]
            exp_v[i] = 3
        else:
            sigs[i] = 0
            sigs[i, 0] = 0xC0
            exp_v[i] = 3
    d["sigs"] = sigs.reshape(-1)
    d["ta_sigs"] = sigs[d["ta_src"]].reshape(-1).copy()
    members = np.asarray(d["ta_src"], dtype=np.int64).reshape(V, t)
    exp_ta = np.zeros(V, dtype=np.uint8)
    exp_agg = np.zeros(V, dtype=np.uint8)
    for v in {i // n for i in cls}:
        mem = [cls.get(int(i)) for i in members[v]]
        if any(c in (0, 1) for c in mem):
            exp_ta[v] = exp_agg[v] = 2
        elif any(c is not None for c in mem):
            exp_agg[v] = 3
    d.update(exp_v=exp_v, exp_ta=exp_ta, exp_agg=exp_agg, n_corrupted=len(cls))


def setup_inputs(L, wl, V, rank):
    """Synthetic cluster -> host arrays; keys and signatures are derived on the GPU."""
    from charon_amd import synth
    from charon_amd.shard import owned_validators
    n, t = wl["n"], wl["t"]
    cl = synth.make_cluster(V, n, t, first_validator=owned_validators(rank, V).start, n_msgs=wl["n_msgs"] or 64,
                            distinct_messages=wl["distinct"])
    NP = V * n
    M = len(cl.msgs)
    msg_of_v = np.asarray(cl.msg_of_validator, dtype=np.uint32)
    midx = np.repeat(msg_of_v, n)
    # the messages are attestation signing roots: M AttestationData (128-byte SSZ, fields from the
    # cluster's synthetic roots) under the attester domain, rooted on the GPU (roots.hip)
    att = attestation_data(cl.msgs, rank)
    domain = attester_domain()
    msgs = np.zeros(32 * M, dtype=np.uint8)
    _chk(L, L.hbls_attestation_signing_roots(_p(att), M, _p(domain), 1, None, _p(msgs)))
    moff = (np.arange(M, dtype=np.uint64) * 32)
    mlen = np.full(M, 32, dtype=np.uint32)
    item_msgs = msgs.reshape(M, 32)[midx].reshape(-1).copy()
    item_off = np.arange(NP, dtype=np.uint64) * 32
    item_len = np.full(NP, 32, dtype=np.uint32)
    sks = np.frombuffer(b"".join(cl.share_sks), dtype=np.uint8).copy()
    pks = np.zeros(NP * 48, dtype=np.uint8)
    sigs = np.zeros(NP * 96, dtype=np.uint8)
    st = np.zeros(NP, dtype=np.uint8)
    _chk(L, L.hbls_secret_to_public_key_batch(_p(sks), NP, _p(pks), _p(st)))
    assert not st.any(), "pubshare derivation failed"
    _chk(L, L.hbls_sign_batch(_p(sks), _p(item_msgs), _p(item_off), _p(item_len), NP, _p(sigs), _p(st)))
    assert not st.any(), "partial signing failed"
    root_sks = np.frombuffer(b"".join(cl.root_sks), dtype=np.uint8).copy()
    root_msgs = msgs.reshape(M, 32)[msg_of_v].reshape(-1).copy()
    root_sigs = np.zeros(V * 96, dtype=np.uint8)
    dv_pks = np.zeros(V * 48, dtype=np.uint8)
    stv = np.zeros(V, dtype=np.uint8)
    root_off = np.arange(V, dtype=np.uint64) * 32  # named: a temporary would be freed before the call
    root_len = np.full(V, 32, dtype=np.uint32)
    _chk(L, L.hbls_sign_batch(_p(root_sks), _p(root_msgs), _p(root_off), _p(root_len), V, _p(root_sigs),
                              _p(stv)))
    assert not stv.any(), "root signing failed"
    _chk(L, L.hbls_secret_to_public_key_batch(_p(root_sks), V, _p(dv_pks), _p(stv)))
    assert not stv.any(), "DV key derivation failed"
    # ThresholdAggregate input: t shares of every validator (parsigdb fires with exactly t,
    # core/parsigdb/memory.go:218-221), given as indices of the verified partials.  The set is
    # that of the t operators whose partials arrived first -- the same for every validator of the
    # duty (parsigex exchanges whole sets per peer), a fixed pseudo-random t-subset here rather
    # than 1..t, whose Lagrange coefficients would be small integers (binomials) and flatter the
    # aggregation ladders
    shares = ta_share_positions(n, t)
    ta_src = (np.arange(V)[:, None] * n + np.asarray(shares)[None, :]).reshape(-1).astype(np.uint32)
    ta_sigs = sigs.reshape(NP, 96)[ta_src].reshape(-1).copy()
    ta_idx = np.tile(np.asarray(shares, dtype=np.int64) + 1, V)
    grp_off = (np.arange(V + 1, dtype=np.uint32) * t)
    vgrp_off = (np.arange(V + 1, dtype=np.uint32) * n)  # one verification group per validator
    return dict(n=n, t=t, V=V, NP=NP, M=M, sks=sks, att=att, domain=domain, msgs=msgs, moff=moff, mlen=mlen, midx=midx, pks=pks, sigs=sigs,
                item_msgs=item_msgs, item_off=item_off, item_len=item_len, ta_sigs=ta_sigs, ta_src=ta_src,
                ta_idx=ta_idx, grp_off=grp_off, vgrp_off=vgrp_off, root_sigs=root_sigs, dv_pks=dv_pks)


def cpu_baseline(d, seconds: float):
    """The host restatement (g++ build of the kernels' per-item arithmetic) on a bounded sample.

    One unit = one validator: n partial Verifies (each hashing its message, as herumi's VerifyByte
    does) + one ThresholdAggregate over t partials, checked against the root-key signature.  The
    loop is native (tests/native/hostcheck.cpp hc_cpu_slot, std::thread workers); threads = usable
    host cores, at most 16."""
    from charon_amd.build import build_hostcheck, check_hostcheck
    hc_path = build_hostcheck(verbose=False)
    hc_id = check_hostcheck(hc_path)  # never time a harness built from other sources
    hc = ctypes.CDLL(hc_path)
    n, t = d["n"], d["t"]
    midx = np.ascontiguousarray(d["midx"], dtype=np.uint32)
    ta_idx = np.ascontiguousarray(d["ta_idx"], dtype=np.int64)  # the aggregated share indices, per validator
    try:
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        threads = max(1, min(16, os.cpu_count() or 1))

    def run(units, th):
        t0 = time.perf_counter()
        bad = hc.hc_cpu_slot(th, units, n, t, _p(d["pks"]), _p(d["sigs"]), _p(d["msgs"]), _p(midx),
                             _p(d["ta_sigs"]), _p(d["root_sigs"]), _p(ta_idx))
        return time.perf_counter() - t0, bad

    per_unit, bad = run(1, 1)
    units = int(min(d["V"], max(threads, seconds * threads / max(per_unit, 1e-6))))
    wall, bad2 = run(units, threads)
    return {"value": round(units * (n + 1) / wall, 2),
            "unit": "items/s (verified partial signatures + ThresholdAggregates)",
            "cores": threads, "kind": "port",
            "sample": f"{units} validators x ({n} partial Verify + 1 ThresholdAggregate of {t}) of the same "
                      f"synthetic cluster; g++ -O3 -march=x86-64-v3 build of the kernels' per-item arithmetic "
                      f"(tests/native/hostcheck.cpp hc_cpu_slot, {threads} std::threads), one hash_to_G2 and one "
                      f"pairing check per Verify as herumi does; not herumi (absent offline), a lower bound on "
                      f"a CPU backend's rate",
            "agrees_with_expected": bad == 0 and bad2 == 0, "wall_s": round(wall, 2),
            "per_core_items_per_s": round(units * (n + 1) / wall / threads, 2),
            "single_thread_items_per_s": round((n + 1) / per_unit, 2),
            "harness_build_id": hc_id}


def concurrent_callers(L, d, threads: int, seconds: float):
    """Unchanged callers: `threads` host threads each calling hbls_verify_batch with ONE item in
    a loop (tbls.Verify from one goroutine per libp2p stream, p2p/receive.go:52); the library
    coalesces them.  Returns single-call latency (idle library) and N-thread throughput."""
    NP = d["NP"]
    pks, sigs, msgs = d["pks"], d["sigs"], d["item_msgs"]
    off0 = np.zeros(1, dtype=np.uint64)
    len32 = np.full(1, 32, dtype=np.uint32)
    lat = []
    for k in range(5):
        st = np.zeros(1, dtype=np.uint8)
        i = (k * 7919) % NP
        t0 = time.perf_counter()
        _chk(L, L.hbls_verify_batch(_p(pks[48 * i:]), _p(sigs[96 * i:]), _p(msgs[32 * i:]), _p(off0), _p(len32), 1,
                                    _p(st)))
        lat.append(time.perf_counter() - t0)
        assert st[0] == 0
    # where one call's time goes: the same call with every launch timed (library timing mode 2:
    # HIP events around each launch, launches serialised)
    _chk(L, L.hbls_timing(2))
    st = np.zeros(1, dtype=np.uint8)
    _chk(L, L.hbls_verify_batch(_p(pks), _p(sigs), _p(msgs), _p(off0), _p(len32), 1, _p(st)))
    single_kern = {}
    for k, ms in _lib_timing(L):
        single_kern[k] = round(single_kern.get(k, 0.0) + ms, 3)
    _chk(L, L.hbls_timing(0))
    stop = time.perf_counter() + seconds
    counts = [0] * threads
    lats = [[] for _ in range(threads)]
    bad = [0]

    def worker(w):
        st = np.zeros(1, dtype=np.uint8)
        k = w
        while time.perf_counter() < stop:
            i = (k * 104729) % NP
            t0 = time.perf_counter()
            rc = L.hbls_verify_batch(_p(pks[48 * i:]), _p(sigs[96 * i:]), _p(msgs[32 * i:]), _p(off0), _p(len32),
                                     1, _p(st))
            lats[w].append(time.perf_counter() - t0)
            if rc != 0 or st[0] != 0:
                bad[0] += 1
            counts[w] += 1
            k += threads

    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(w,)) for w in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    wall = time.perf_counter() - t0
    all_l = [x for l in lats for x in l]
    return {"threads": threads, "calls_per_s": round(sum(counts) / wall, 1),
            "mean_latency_ms": round(1e3 * statistics.mean(all_l), 2) if all_l else None,
            "single_call_latency_ms": round(1e3 * statistics.median(lat), 2), "all_ok": bad[0] == 0,
            "single_call_kernels_ms": single_kern,
            "coalesce_us": int(os.environ.get("HBLS_COALESCE_US", "200"))}


R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def aggregate_verify(L, d, d_pk, dev, sp, reps: int = 3, sync_size: int = 512):
    """VerifyAggregate at scale on the resident pubshares (hbls_verify_aggregate_device):
      lock: ONE group of all V*n public shares against a lock hash (cluster/lock.go:185, run at
            every charon start over every validator's every pubshare);
      sync: groups of 512 public keys, each over its own message (sync-committee aggregate,
            BASELINE configs[4]), message hashing included.
    The signatures are sum(sk) * H(m), produced once by hbls_sign_batch outside the timed region."""
    import hashlib
    import torch
    NP, sks = d["NP"], d["sks"]
    ints = [int.from_bytes(sks[32 * i:32 * i + 32].tobytes(), "big") for i in range(NP)]
    G = NP // sync_size
    sums = [sum(ints) % R_ORDER] + [sum(ints[g * sync_size:(g + 1) * sync_size]) % R_ORDER for g in range(G)]
    msgs = [hashlib.sha256(b"cluster lock hash").digest()] + \
        [hashlib.sha256(b"sync committee root %d" % g).digest() for g in range(G)]
    m = np.frombuffer(b"".join(msgs), dtype=np.uint8).copy()
    moff = np.arange(G + 1, dtype=np.uint64) * 32
    mlen = np.full(G + 1, 32, dtype=np.uint32)
    sk_b = np.frombuffer(b"".join(x.to_bytes(32, "big") for x in sums), dtype=np.uint8).copy()
    sigs = np.zeros(96 * (G + 1), dtype=np.uint8)
    st = np.zeros(G + 1, dtype=np.uint8)
    _chk(L, L.hbls_sign_batch(_p(sk_b), _p(m), _p(moff), _p(mlen), G + 1, _p(sigs), _p(st)))
    assert not st.any()
    up = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    d_m, d_mo, d_ml, d_sig = up(m), up(moff.view(np.int64)), up(mlen.view(np.int32)), up(sigs)
    d_hm = torch.zeros((G + 1) * L.hbls_hm_entry_bytes(), dtype=torch.uint8, device=dev)
    d_st = torch.full((G + 1,), 255, dtype=torch.uint8, device=dev)
    lock_off = np.array([0, NP], dtype=np.uint32)
    sync_off = np.arange(G + 1, dtype=np.uint32) * sync_size
    spp = sp
    hm_sz = L.hbls_hm_entry_bytes()

    def lock():
        _chk(L, L.hbls_hash_to_g2_device(_p(d_m), _p(d_mo), _p(d_ml), 1, _p(d_hm), spp))
        _chk(L, L.hbls_verify_aggregate_device(_p(d_pk), _p(lock_off), 1, _p(d_sig), _p(d_hm), _p(d_st), spp))

    def sync():
        hm1 = ctypes.c_void_p(d_hm.data_ptr() + hm_sz)
        _chk(L, L.hbls_hash_to_g2_device(ctypes.c_void_p(d_m.data_ptr() + 32), _p(d_mo[:G]), _p(d_ml[:G]), G, hm1,
                                         spp))
        _chk(L, L.hbls_verify_aggregate_device(_p(d_pk), _p(sync_off), G, ctypes.c_void_p(d_sig.data_ptr() + 96),
                                               hm1, ctypes.c_void_p(d_st.data_ptr() + 1), spp))

    out = {}
    for name, fn, units in (("lock", lock, 1), ("sync_committee", sync, G)):
        fn()  # warm-up (workspace growth)
        torch.cuda.synchronize(dev)
        _chk(L, L.hbls_timing(1))
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        wall = (time.perf_counter() - t0) / reps
        recs = _lib_timing(L)
        _chk(L, L.hbls_timing(0))
        stv = d_st.cpu().numpy()
        ok = bool(stv[0] == 0) if name == "lock" else bool((stv[1:] == 0).all())
        kern = {}
        for k, ms in recs:
            kern[k] = round(kern.get(k, 0.0) + ms / reps, 3)
        per_group = NP if name == "lock" else sync_size
        dec_ms = kern.get("k_dec_pk")
        dec_tops = (units * per_group * opcounts.BLOCKS["g1_dec"] * opcounts.MAC_PER_FPMUL / (dec_ms * 1e-3) / 1e12
                    if dec_ms else None)
        out[name] = {"groups": units, "keys_per_group": per_group, "ms": round(wall * 1e3, 3),
                     "keys_per_s": round(units * per_group / wall, 1), "all_ok": ok, "kernel_ms": kern,
                     "k_dec_pk_Tops_alg": round(dec_tops, 3) if dec_tops else None,
                     "k_dec_pk_frac": round(dec_tops / opcounts.PEAK_MAD_TOPS, 4) if dec_tops else None}
    return out


def first_error_verify(L, d, d_pk, d_sig, d_midx, d_vgoff, dev, sp, reps: int = 3):
    """The corrupted shard's partials as ONE ordered set verified up to its first failure
    (hbls_verify_device_first_error: the callers' first-error-aborts contract, parsigex.go:93-98,
    sigagg.go:56-63) beside the exact per-item verdicts of the same items (hbls_verify_device),
    hashing included in both; the first index is checked against the construction."""
    import torch
    NP, M = d["NP"], d["M"]
    up = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    d_m, d_mo, d_ml = up(d["msgs"]), up(d["moff"].view(np.int64)), up(d["mlen"].view(np.int32))
    hm = torch.zeros(M * L.hbls_hm_entry_bytes(), dtype=torch.uint8, device=dev)
    st = torch.full((NP,), 255, dtype=torch.uint8, device=dev)
    first = torch.zeros(1, dtype=torch.int32, device=dev)
    V = d["V"]

    def run(first_mode):
        _chk(L, L.hbls_hash_to_g2_device(_p(d_m), _p(d_mo), _p(d_ml), M, _p(hm), sp))
        if first_mode:
            _chk(L, L.hbls_verify_device_first_error(_p(d_pk), _p(d_sig), _p(d_midx), _p(hm), NP, _p(d_vgoff), V,
                                                     _p(st), _p(first), sp))
        else:
            _chk(L, L.hbls_verify_device(_p(d_pk), _p(d_sig), _p(d_midx), _p(hm), NP, _p(d_vgoff), V, _p(st), sp))

    res = {}
    for mode in (True, False):
        run(mode)  # warm-up
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            run(mode)
        torch.cuda.synchronize(dev)
        res[mode] = (time.perf_counter() - t0) / reps
    run(True)
    torch.cuda.synchronize(dev)
    f = int(first.cpu().numpy().view(np.uint32)[0])
    bad = np.nonzero(d["exp_v"] != 0)[0]
    want = int(bad[0]) if len(bad) else 0xFFFFFFFF
    stv = st.cpu().numpy()
    return {"items": NP, "ms": round(res[True] * 1e3, 3), "items_per_s": round(NP / res[True], 1),
            "exact_ms": round(res[False] * 1e3, 3), "exact_items_per_s": round(NP / res[False], 1),
            "first_index": f, "first_index_exact": bool(f == want and (f == 0xFFFFFFFF or stv[f] == d["exp_v"][f])),
            "unchecked_items": int((stv == 7).sum()),
            "note": "hash + verify of the shard's partials as one ordered set, first-error mode against "
                    "exact per-item statuses (no aggregation)"}


def key_table_slots(L, d_pk, d_dvpk, outs, NP, V, steps, step, mk, items):
    """The same slots with the public keys taken from decompressed-key tables made once
    (hbls_decompress_pubkeys_device; pubshares are static per cluster lock): the
    steady state of a node, reported beside the headline, which decompresses every key."""
    import torch
    E = L.hbls_pk_entry_bytes()
    dev = d_pk.device
    tab = torch.zeros(NP * E, dtype=torch.uint8, device=dev)
    tst = torch.full((NP,), 255, dtype=torch.uint8, device=dev)
    dtab = torch.zeros(V * E, dtype=torch.uint8, device=dev)
    dst = torch.full((V,), 255, dtype=torch.uint8, device=dev)
    s0 = ctypes.c_void_p(outs[0]["stream"].cuda_stream)
    t0 = time.perf_counter()
    _chk(L, L.hbls_decompress_pubkeys_device(_p(d_pk), NP, _p(tab), _p(tst), s0))
    _chk(L, L.hbls_decompress_pubkeys_device(_p(d_dvpk), V, _p(dtab), _p(dst), s0))
    torch.cuda.synchronize()
    build_ms = (time.perf_counter() - t0) * 1e3
    for o in outs:
        o["slot"].pk_table, o["slot"].pk_table_st = _p(tab).value, _p(tst).value
        o["slot"].dv_pk_table, o["slot"].dv_pk_table_st = _p(dtab).value, _p(dst).value
    for _ in range(len(outs)):  # every in-flight output set once with the tables (warm-up)
        step(mk())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(mk())
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    ok = all(bool((o["vst"] == 0).all().item()) and bool((o["tst"] == 0).all().item()) and
             bool((o["ast"] == 0).all().item()) for o in outs)
    for o in outs:
        o["slot"].pk_table = o["slot"].pk_table_st = o["slot"].dv_pk_table = o["slot"].dv_pk_table_st = None
    return {"items_per_s": round(items / el, 1), "ms_per_step": round(el * 1e3, 3), "steps": steps,
            "table_build_ms": round(build_ms, 3), "all_ok": ok}


def _lib_timing(L):
    from charon_amd import _lib
    return _lib.timing_read(L)


def valu_issue_of(kernel, ms_alone, n_cu):
    """The dominant kernel against the VALU ISSUE ceiling: its wave-level VALU instructions per slot
    (SQ_INSTS_VALU, committed PMC pass of this build, profiles/pmc_traffic.json) over its alone time,
    against one wave instruction per SIMD per 4 clocks (n_cu x 4 SIMDs x clock / 4) at the peak's
    measured clock.  v_mad_u64_u32 itself issues at 0.84 of that (profiles/r05b_peak_from_counters.json)."""
    try:
        k = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))["kernels"].get(kernel)
    except (OSError, ValueError, KeyError):
        return None
    if not k or not k.get("valu_wave_insts") or not ms_alone:
        return None
    ceil = n_cu * opcounts.PEAK_CLOCK_MHZ * 1e6  # wave instructions / s
    got = k["valu_wave_insts"] / (ms_alone * 1e-3)
    return {"wave_insts_per_step": k["valu_wave_insts"], "achieved_G_per_s": round(got / 1e9, 1),
            "ceiling_G_per_s": round(ceil / 1e9, 1), "frac": round(got / ceil, 4),
            "mad_issue_frac_of_ceiling": round(opcounts.PEAK_MAD_TOPS / (n_cu * 64 * opcounts.PEAK_CLOCK_MHZ * 1e-6), 4),
            "source": "profiles/pmc_traffic.json valu_wave_insts (SQ_INSTS_VALU of the PMC pass)"}


def slot_valu_insts():
    """Wave-level VALU instructions of one C3 slot, summed over the timed kernel labels of the
    committed PMC pass (profiles/pmc_traffic.json), or None."""
    try:
        ks = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    return sum(k.get("valu_wave_insts", 0) for k in ks.values()) or None


def slot_issue(workload, step_s, n_cu):
    """C3 only (the PMC pass is of a C3 slot): the slot's VALU instructions over the measured step
    time against the issue ceiling (one wave instruction per SIMD per 4 clocks)."""
    n = slot_valu_insts() if workload == "c3" else None
    if not n:
        return {}
    return {"valu_wave_insts_per_step": n,
            "valu_issue_frac": round(n / step_s / (n_cu * opcounts.PEAK_CLOCK_MHZ * 1e6), 4)}


def traffic_of(kernel):
    """HBM bytes per slot of `kernel` (all its launches, FETCH_SIZE x2 + WRITE_SIZE) from the
    committed PMC pass, or None (rocprofv3 counters cannot be read from inside the timed run)."""
    try:
        k = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))["kernels"].get(kernel)
        return round(k["bytes_per_slot"]) if k else None
    except (OSError, ValueError, KeyError):
        return None


def roofline_from_timing(recs, steps, units):
    """Per-kernel totals over the timed steps; the dominant kernel's roofline entry."""
    tot, cnt = {}, {}
    for name, ms in recs:
        tot[name] = tot.get(name, 0.0) + ms
        cnt[name] = cnt.get(name, 0) + 1
    per = {}
    for name in tot:
        if name not in units:
            continue
        u, (alg, exe) = units[name]
        t = tot[name] / steps * 1e-3  # s per step
        per[name] = {"ms_per_step": round(tot[name] / steps, 3), "launches_per_step": cnt[name] / steps,
                     "units_per_step": u, "fpmul_per_unit_alg": alg, "fpmul_per_unit_exec": exe,
                     "achieved_Tops_alg": round(u * alg * opcounts.MAC_PER_FPMUL / t / 1e12, 3) if t > 0 else None,
                     "achieved_Tops_exec": round(u * exe * opcounts.MAC_PER_FPMUL / t / 1e12, 3) if t > 0 else None}
    # the dominant kernel: the most algorithmic work per step (the longest alone time can be a
    # latency-bound kernel with little work, e.g. the hashing of C2's 64 messages)
    dom = max(per, key=lambda k: per[k]["units_per_step"] * per[k]["fpmul_per_unit_alg"]) if per else None
    return dom, per


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` without a launcher: run N ranks of this script as child processes, one
    per GPU, with the environment torch.distributed.run would give them (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR 127.0.0.1, a free MASTER_PORT).  This process never touches the GPU: it
    starts the children, forwards nothing (they share its stdout, where rank 0 prints the one JSON
    line), and returns the first failing child's exit status -- stopping the others, which would
    otherwise wait at a barrier for the rank that died."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                      file=sys.stderr)
                for q in live:
                    q.terminate()
                for q in live:
                    try:
                        q.wait(timeout=20)
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                live = []
        time.sleep(0.05)
    return rc


def keep_stdout_for_the_line() -> None:
    """Stdout carries only rank 0's JSON line.  Native libraries write to file descriptor 1 of every
    rank (gloo prints "[Gloo] Rank r is connected to ..." when a group forms, under
    torch.distributed.run on the launcher's shared stdout): point descriptor 1 at stderr and give
    Python's sys.stdout a stream on the original descriptor, which only the line is printed to."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    sys.stdout = os.fdopen(fd, "w", buffering=1)


def dry_run(args, rank: int, world: int, local: int) -> int:
    """The launcher and the control plane without a GPU: every rank joins gloo, the ranks' own
    environments and a stand-in step time are gathered, rank 0 prints the merged line."""
    import torch.distributed as dist
    if args.dry_run == 2 and rank == world - 1:  # the launcher test's failing rank
        print(f"rank {rank}: failing on purpose (--dry-run 2)", file=sys.stderr)
        return 3
    mine = {"rank": rank, "local_rank": local, "world_size": world,
            "master_addr": os.environ.get("MASTER_ADDR"), "master_port": os.environ.get("MASTER_PORT"),
            "pid": os.getpid()}
    t0 = time.perf_counter()
    sum(i * i for i in range(20000 * (rank + 1)))
    el = time.perf_counter() - t0
    envs, times = [mine], [el]
    if world > 1:
        dist.init_process_group("gloo")
        envs, times = [None] * world, [None] * world
        dist.all_gather_object(envs, mine)
        dist.all_gather_object(times, el)
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "dry_run": True, "ranks": envs,
                          "per_rank_ms_per_step": [round(x * 1e3, 3) for x in times],
                          "ms_per_step": round(max(times) * 1e3, 3)}), flush=True)
    return 0


def main(argv=None):
    ap = argparse.ArgumentParser(description="charon BLS hot path on MI355X")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--validators", type=int, default=0, help="override validators per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample (0: skip)")
    ap.add_argument("--callers", type=int, default=64, help="threads of the concurrent-caller measurement (0: skip)")
    ap.add_argument("--callers-seconds", type=float, default=4.0)
    ap.add_argument("--aggregate-verify", type=int, default=1,
                    help="also time VerifyAggregate at scale (lock over all pubshares, sync-committee groups)")
    ap.add_argument("--key-tables", type=int, default=1,
                    help="also time the slot with decompressed-key tables built once (steady state)")
    ap.add_argument("--host-api", type=int, default=1,
                    help="also time the host-buffer (PCIe-inclusive) entry points on the same inputs (0: skip)")
    ap.add_argument("--bad-frac", type=float, default=None,
                    help="fraction of the partials corrupted in equal fifths (bench.corrupt; default: the "
                         "workload's, 0.01 for c5) -- the attack curve: c5 at 0.01 / 0.05 / 0.10")
    ap.add_argument("--host-runs", type=int, default=3,
                    help="timed runs of the host-buffer pair after one warm-up (the median is reported)")
    ap.add_argument("--host-threads", type=int, default=3,
                    help="threads calling the host-buffer entry points at once (with --host-api; 1: skip)")
    ap.add_argument("--inflight", type=int, default=3,
                    help="slots in flight (each on its own stream and outputs); 1 = one slot at a time")
    ap.add_argument("--exchange-rehearsal", type=int, default=0,
                    help="at one GPU: run the multi-GPU exchange (RCCL world of one) inside the timed region")
    ap.add_argument("--mode", default="slot", choices=["slot", "staged"],
                    help="slot: one hbls_slot_device call per step (stages overlap); staged: stage by stage")
    ap.add_argument("--share-device", type=int, default=0,
                    help="rehearsal of the N > 1 path on a one-GPU box: every rank on device 0, the slot "
                         "exchange over gloo through host copies (RCCL refuses two ranks on one GPU); the line "
                         "is marked rehearsal and is not a measurement")
    ap.add_argument("--dry-run", type=int, default=0,
                    help="1: no GPU -- every rank joins the gloo control plane, reports its rank environment "
                         "and prints the merged line (tests the launcher on a CPU host); 2: the same with "
                         "the last rank failing")
    args = ap.parse_args(argv)

    if args.gpus < 1:
        print(f"bench.py: --gpus {args.gpus}: need at least one", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start the N ranks here, before anything in this process touches the GPU
        return launch_ranks(args.gpus, sys.argv[1:] if argv is None else list(argv))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", rank))
    if world != args.gpus:
        # never measure a world other than the one asked for (a line labelled with the wrong N)
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}: refusing to run", file=sys.stderr)
        return 2
    keep_stdout_for_the_line()
    if args.dry_run:
        return dry_run(args, rank, world, local)

    import torch
    import torch.distributed as dist
    from charon_amd.shard import (SlotExchange, init_library_comm, library_allgather, max_over_ranks,
                                   pack_layout, pack_views, unpack_gathered)

    if args.share_device:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("gloo")  # control plane only: the slot exchange is the library's RCCL

    from charon_amd import _lib
    L = _lib.load_library()
    _chk(L, L.hbls_init(1 << local))

    wl = WORKLOADS[args.workload]
    V = args.validators or wl["validators"]
    d = setup_inputs(L, wl, V, rank)
    bad_frac = args.bad_frac if args.bad_frac is not None else wl.get("adversarial", 0.0)
    if bad_frac:
        corrupt(L, d, bad_frac, seed=7 + rank)
    n, t, NP, M = d["n"], d["t"], d["NP"], d["M"]
    dev = torch.device("cuda", local)

    def up(a):
        return torch.from_numpy(a).to(dev)

    d_msg, d_moff, d_mlen = up(d["msgs"]), up(d["moff"].view(np.int64)), up(d["mlen"].view(np.int32))
    d_att, d_dom = up(d["att"]), up(d["domain"])
    d_midx, d_pk, d_sig = up(d["midx"].view(np.int32)), up(d["pks"]), up(d["sigs"])
    d_tsrc, d_tidx, d_goff = up(d["ta_src"].view(np.int32)), up(d["ta_idx"]), up(d["grp_off"].view(np.int32))
    d_vgoff, d_dvpk, d_tsig = up(d["vgrp_off"].view(np.int32)), up(d["dv_pks"]), up(d["ta_sigs"])
    # per in-flight slot: its own stream, hashed-message table and outputs (inputs are shared)
    n_sets = max(1, args.inflight)
    # what the ranks exchange lives in ONE buffer per slot -- [verify bitmap | aggregates | their
    # statuses | the aggregates' verification statuses] -- that the slot writes in place, so a slot
    # takes one all-gather (each RCCL call costs ~1 ms of latency however small)
    PACK, PB = pack_layout(NP, V)
    NB = PACK["vbits"][1]

    def out_set():
        o = {"hm": torch.zeros(M * L.hbls_hm_entry_bytes(), dtype=torch.uint8, device=dev),
             "vst": torch.full((NP,), 255, dtype=torch.uint8, device=dev),
             "pack": torch.zeros(PB, dtype=torch.uint8, device=dev),
             "msg": torch.zeros(M * 32, dtype=torch.uint8, device=dev),
             "stream": torch.cuda.Stream(device=dev)}
        o.update(pack_views(o["pack"], PACK))
        o["tst"].fill_(255)
        o["ast"].fill_(255)
        return o

    outs = [out_set() for _ in range(n_sets)]
    d_hm, d_vst, d_tout, d_tst, d_ast = (outs[0][k] for k in ("hm", "vst", "tout", "tst", "ast"))

    xchg = None
    exch = None
    xw = world > 1 or bool(args.exchange_rehearsal)  # the exchange runs (a world of one: a rehearsal)
    if xw:
        # the library's RCCL communicator (rank 0's id over the gloo control plane), then ONE
        # exchange stream for the all-gathers of every in-flight slot (charon_amd/shard.py
        # SlotExchange: the same ordering code tests/test_shard.py runs over gloo)
        if args.share_device:
            def host_allgather(send, recv, nbytes, stream):  # the rehearsal's stand-in for RCCL
                stream.synchronize()  # the producer's outputs (the exchange stream waited for them)
                hr = torch.empty(world * nbytes, dtype=torch.uint8)
                dist.all_gather_into_tensor(hr, send.cpu())
                with torch.cuda.stream(stream):
                    recv.copy_(hr.to(dev))
            allgather = host_allgather
        else:
            init_library_comm(L, world, rank)
            allgather = library_allgather(L)
        exch = SlotExchange(world, rank, {"pack": PB}, dev, allgather, stream=torch.cuda.Stream(device=dev))
        for o in outs:
            o["xchg"] = exch.gather_buffers()
        xchg = outs[0]["xchg"]

    def gathered(f):  # field f of every rank, in rank order, from the gathered packs
        return unpack_gathered(xchg["pack"], PACK, PB, world, f)

    stream = outs[0]["stream"]
    sp = ctypes.c_void_p(stream.cuda_stream)
    for o in outs:
        o["sp"] = ctypes.c_void_p(o["stream"].cuda_stream)
        o["slot"] = _lib.HblsSlot(
            msgs=_p(o["msg"]).value, msg_off=_p(d_moff).value, msg_len=_p(d_mlen).value, n_msgs=M, hm=_p(o["hm"]).value,
            pks=_p(d_pk).value, sigs=_p(d_sig).value, msg_idx=_p(d_midx).value, n=NP, vgrp_off=_p(d_vgoff).value,
            n_vgroups=V, vstatus=_p(o["vst"]).value, ta_sigs=None, ta_src=_p(d_tsrc).value, ta_idx=_p(d_tidx).value,
            grp_off=_p(d_goff).value, n_groups=V, n_ta_partials=V * t, ta_out=_p(o["tout"]).value,
            ta_status=_p(o["tst"]).value, dv_pks=_p(d_dvpk).value, agg_vstatus=_p(o["ast"]).value)

    def exchange(o):  # all-gather verify bitmaps + compressed aggregates to every rank (RCCL)
        _chk(L, L.hbls_status_bitmap(_p(o["vst"]), NP, _p(o["vbits"]), o["sp"]))
        exch.exchange({"pack": o["pack"]}, o["xchg"], producer=o["stream"])

    step_no = [0]

    def step_slot(ev):
        # consecutive slots alternate between the in-flight sets: slot k+1's decompression and
        # hashing run while slot k's pairings finish (the library orders its workspaces by events)
        o = outs[step_no[0] % n_sets]
        step_no[0] += 1
        st = o["stream"]
        ev[0].record(st)
        # the slot's messages: attestation signing roots from the SSZ AttestationData (§8(f)3)
        _chk(L, L.hbls_attestation_signing_roots_device(_p(d_att), M, _p(d_dom), 1, None, _p(o["msg"]), o["sp"]))
        _chk(L, L.hbls_slot_device(ctypes.byref(o["slot"]), o["sp"]))
        ev[1].record(st)
        if xw:
            exchange(o)
        ev[2].record(st)

    def step_staged(ev):
        # the same work stage by stage (no overlap; the aggregation decompresses its own bytes)
        ev[0].record(stream)
        _chk(L, L.hbls_hash_to_g2_device(_p(d_msg), _p(d_moff), _p(d_mlen), M, _p(d_hm), sp))
        ev[1].record(stream)
        _chk(L, L.hbls_verify_device(_p(d_pk), _p(d_sig), _p(d_midx), _p(d_hm), NP, _p(d_vgoff), V, _p(d_vst), sp))
        ev[2].record(stream)
        _chk(L, L.hbls_threshold_aggregate_device(_p(d_tsig), _p(d_tidx), _p(d_goff), V, V * t, _p(d_tout),
                                                  _p(d_tst), sp))
        ev[3].record(stream)

    staged = args.mode == "staged"
    step = step_staged if staged else step_slot
    n_ev = 4 if staged else 3

    def mk():
        return [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]

    for _ in range(args.warmup):
        step(mk())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # no per-launch event instrumentation inside the timed region (the per-kernel figures come
    # from the serialised slot after it); HBLS_BENCH_TIMED_EVENTS=1 keeps it on, for comparison
    timed_events = os.environ.get("HBLS_BENCH_TIMED_EVENTS") == "1"
    if timed_events:
        _chk(L, L.hbls_timing(1))
    evs = [mk() for _ in range(args.steps)]
    PACE = os.environ.get("HBLS_BENCH_PACE", "1") != "0"
    t0 = time.perf_counter()
    for k in range(args.steps):
        # slot k is enqueued once slot k - n_sets (the one before it on its stream) has completed,
        # as a node takes slots as they come, rather than every slot up front (HBLS_BENCH_PACE=0):
        # 12.79-12.84 against 12.59-12.68 M items/s at 20 steps on one box (profiles/r05af_*)
        if PACE and k >= n_sets:
            evs[k - n_sets][-1].synchronize()
        step(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per_rank_s = [elapsed]
    if world > 1:
        per_rank_s = [None] * world
        dist.all_gather_object(per_rank_s, elapsed)
        elapsed = max_over_ranks(elapsed, torch.device("cpu"))

    seg = np.array([[e[i].elapsed_time(e[i + 1]) for i in range(n_ev - 1)] for e in evs])  # ms
    k_ms = seg.mean(axis=0)
    if timed_events:
        _chk(L, L.hbls_timing(0))

    # parity of the timed outputs: every partial verifies, every aggregate is byte-identical to the
    # root-key signature (tbls_test.go:72-97 property) and verifies under the DV key
    # the output sets the timed steps wrote (a short run may leave some of the in-flight sets unused)
    used = [outs[k % n_sets] for k in sorted({k % n_sets for k in range(args.warmup, args.warmup + args.steps)})] \
        if not staged else outs[:1]
    if "exp_v" in d:  # C5: every status bit-exact against construction
        clean = d["exp_agg"] == 0
        parity = {"verify_statuses_exact": all(np.array_equal(o["vst"].cpu().numpy(), d["exp_v"]) for o in used),
                  "ta_statuses_exact": all(np.array_equal(o["tst"].cpu().numpy(), d["exp_ta"]) for o in used),
                  "ta_equals_root_signature_where_clean": all(np.array_equal(
                      o["tout"].cpu().numpy().reshape(V, 96)[clean], d["root_sigs"].reshape(V, 96)[clean])
                      for o in used)}
        if not staged:
            parity["aggregate_verify_statuses_exact"] = all(
                np.array_equal(o["ast"].cpu().numpy(), d["exp_agg"]) for o in used)
    else:
        parity = {"verify_all_ok": all(bool((o["vst"] == 0).all().item()) for o in used),
                  "ta_all_ok": all(bool((o["tst"] == 0).all().item()) for o in used),
                  "ta_equals_root_signature": all(np.array_equal(o["tout"].cpu().numpy(), d["root_sigs"])
                                                  for o in used)}
        if not staged:
            parity["aggregate_verify_all_ok"] = all(bool((o["ast"] == 0).all().item()) for o in used)
    if xw and "exp_v" in d:  # every rank's block equals that rank's construction: check our own
        parity["allgather_ok"] = bool(
            np.array_equal(gathered("vbits")[rank * NB:(rank + 1) * NB].cpu().numpy(),
                           np.packbits(d["exp_v"] == 0, bitorder="little")) and
            np.array_equal(gathered("tst")[rank * V:(rank + 1) * V].cpu().numpy(), d["exp_ta"]) and
            np.array_equal(gathered("ast")[rank * V:(rank + 1) * V].cpu().numpy(), d["exp_agg"]))
    elif xw:
        want = torch.from_numpy(np.packbits(np.ones(NP, dtype=bool), bitorder="little")).to(dev)
        gv = gathered("vbits")
        parity["allgather_ok"] = bool(all(torch.equal(gv[r * NB:(r + 1) * NB], want) for r in range(world))
                                      and (gathered("tst") == 0).all().item() and (gathered("ast") == 0).all().item())
        # rank r's block of the gathered aggregates is rank r's root signatures: check our own block
        clean = d["exp_agg"] == 0 if "exp_v" in d else np.ones(V, dtype=bool)
        parity["allgather_own_block"] = bool(np.array_equal(
            gathered("tout")[rank * V * 96:(rank + 1) * V * 96].cpu().numpy().reshape(V, 96)[clean],
            d["root_sigs"].reshape(V, 96)[clean]))

    items = world * (NP + V)
    ms_per_step = elapsed / args.steps * 1e3
    value = items / (elapsed / args.steps)

    def kernel_roofline():
        # per-kernel roofline: the same slot once more with every kernel ALONE on the device
        # (timing mode 2 serialises the launches), after every other measurement -- overlapped
        # launches of the slots in flight share the chip and their durations say nothing about one
        # kernel; as the last slot of the run it is also the last one in a rocprofv3 trace
        torch.cuda.synchronize()
        _chk(L, L.hbls_timing(2))
        step(mk())
        torch.cuda.synchronize()
        recs = _lib.timing_read(L)
        _chk(L, L.hbls_timing(0))
        per_unit = opcounts.per_unit(group_size=n, t=t)
        ta_units = V * t
        jc_knob = L.hbls_ta_joint(0)
        L.hbls_ta_joint(jc_knob)
        # k_rlc: the partials as multi-scalar chunks (one per validator), then the folded
        # aggregates (slot mode)
        # batched final exponentiation (the library's setting; verifications of >= fe_min groups):
        # every folded aggregate then takes a random coefficient (one ladder each), else r = 1
        fe_min = L.hbls_fe_batch(0)
        L.hbls_fe_batch(fe_min)
        bfe = fe_min and V >= fe_min
        # slot-wide check (the library's setting): the signature side as one MSM, so the
        # combination kernels compute the public-key side only
        s_min = L.hbls_slot_msm(0)
        L.hbls_slot_msm(s_min)
        n_rlc = NP + (0 if staged else V)
        # (C5: the slot-wide check fails on the corrupted partials and the per-batch, per-group and
        # per-item checks run behind it -- data-dependent work: the kernels that only they launch, or
        # share with the slot-wide check, are listed with zero units; k_rlc counts both sides)
        smsm = bool(bfe and s_min and n_rlc >= s_min)
        fallback = "exp_v" in d
        sides = 1 if smsm and not fallback else 3
        rlc_item = opcounts.BLOCKS["rlc_g1"] + (opcounts.BLOCKS["rlc_g2"] if sides & 2 else 0)
        cmax = min(opcounts.RLC_CHUNK, max(1, NP // int(os.environ.get("HBLS_RLC_LANES", "65536"))))
        if cmax > 1:  # the library's chunking (hipbls.hip verify_pipeline): balanced chunks of a group
            n_chunks = -(-n // cmax)
            rlc_partial = opcounts.rlc_msm(chunk=n / n_chunks, sides=sides)
        else:
            rlc_partial = rlc_item
        rlc_avg = (NP * rlc_partial + (0 if staged or not bfe else V * rlc_item)) / n_rlc
        ta_ids = [x + 1 for x in ta_share_positions(n, t)]
        jc = opcounts.ta_joint_chunk(t, ta_units, jc_knob)
        ta_w = opcounts.ta_joint(ta_ids, jc) if jc else opcounts.ta_uniform(ta_ids)
        # the small-scalar aggregation (threshold.hip k_ta_small, one lane per validator) takes every
        # group whose index set it can split; the per-member ladders then have nothing to do
        ta_small_w = opcounts.ta_small(ta_ids)
        prep_units = opcounts.per_unit(group_size=n + (0 if staged else 1), t=t)
        units = {"k_rlc": (n_rlc, (rlc_avg, rlc_avg)),
                 "k_dec_pk": (NP + (0 if staged else V), per_unit["k_dec_pk"]),
                 "k_dec_sig_pt": (NP + (ta_units if staged else 0), per_unit["k_dec_sig_pt"]),
                 # the aggregation ladders: the uniform-digit schedule of the aggregated index set
                 "k_ta_straus": (0 if ta_small_w else ta_units, (ta_w, ta_w)),
                 "k_ta_small": (V if ta_small_w else 0, (ta_small_w or 0, ta_small_w or 0)),
                 "k_group_sum": (V, per_unit["k_group_sum"]),
                 "k_hash_to_g2": (M, per_unit["k_hash_to_g2"]), "k_lines_msg": (M, per_unit["k_lines_msg"])}
        if smsm:
            # multi-Miller loops of MML_PAIRS groups, product tree of fan-in FE_BATCH to <= FE_BATCH
            n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
            mmlk = opcounts.mml_pairs(V, n_cu)
            n_prod = opcounts.prod_tree_inputs(-(-V // mmlk))
            fin = opcounts.pair3_fin(batch=2, lines=False)
            units.update({"k_group_prep": (V, prep_units["k_group_prep_p"]),
                          # the signature side's lines and loop in one kernel (k_lml)
                          "k_pair3_mls": (1, tuple(a + b for a, b in zip(per_unit["k_pair3_mls"], per_unit["k_slines"]))),
                          "k_pair3_mml": (V, opcounts.pair3_mml(pairs=mmlk)),
                          "k_mml_eval": (V, per_unit["k_mml_eval"]),
                          "k_lines_at_p": (0, per_unit["k_lines_at_p"]),
                          "k_pair3_prod": (n_prod, per_unit["k_pair3_prod"]),
                          "k_pair3_fin": (1, fin), "k_slines": (1, per_unit["k_slines"]),
                          "k_msm_bucket": (opcounts.MSM_ENTRIES_PER_ITEM * n_rlc, per_unit["k_msm_bucket"]),
                          "k_msm_reduce": (opcounts.MSM_PARTS, per_unit["k_msm_reduce"]),
                          "k_msm_sum": (opcounts.MSM_PARTS + opcounts.MSM_PARTS // 128, per_unit["k_msm_sum"])})
            if M >= V and not fallback:
                # distinct messages, one group each (hipbls.hip defer_lines): the chains evaluated at
                # P by k_lines_at_p; the unevaluated lines only behind a failed check (k_lines_msg
                # guarded, k_mml_eval not launched)
                units["k_lines_at_p"] = (V, per_unit["k_lines_at_p"])
                units["k_lines_msg"] = (0, per_unit["k_lines_msg"])
                units["k_mml_eval"] = (0, per_unit["k_mml_eval"])
            if fallback:
                for kname in ("k_group_prep", "k_pair3_fin", "k_slines", "k_pair3_ml", "k_pair3_fallback", "k_fb_lines"):
                    units[kname] = (0, units.get(kname, (0, (0, 0)))[1])
        elif bfe:
            nb = -(-V // opcounts.FE_BATCH)
            units.update({"k_group_prep": (V, prep_units["k_group_prep_b"]),
                          "k_pair3_ml": (V, per_unit["k_pair3_ml"]), "k_pair3_fin": (nb, per_unit["k_pair3_fin"]),
                          "k_pair3_mls": (nb, per_unit["k_pair3_mls"]),
                          "k_pair3_prod": (V + -(-V // opcounts.PROD_FAN), per_unit["k_pair3_prod"]),
                          "k_slines": (nb, per_unit["k_slines"])})
        else:
            units.update({"k_group_prep": (V, prep_units["k_group_prep"]), "k_pair3": (V, per_unit["k_pair3"])})
        dom, per = roofline_from_timing(recs, 1, units)
        # the whole slot: every kernel's algorithmic work over the measured step time
        slot_fpmul = sum(u * w[0] for u, w in units.values())
        slot_tops = slot_fpmul * opcounts.MAC_PER_FPMUL / (elapsed / args.steps) / 1e12
        pair = per.get("k_pair3") or {k: per.get(k) for k in ("k_pair3_ml", "k_pair3_fin")}
        roofline = None
        if dom:
            x = per[dom]
            roofline = {"bound": "valu", "kernel": dom, "unit_of_work": opcounts.UNITS.get(dom),
                        "achieved": x["achieved_Tops_alg"], "peak": opcounts.PEAK_MAD_TOPS,
                        "unit": "Tops/s (32-bit multiply-add lane-ops, v_mad_u64_u32)",
                        # the peak: measured (16 waves/CU, event-timed, counters agree), the clock
                        # it ran at, and the architectural issue bound at the nominal clock
                        "peak_measured": opcounts.PEAK_MAD_TOPS, "peak_nominal": opcounts.PEAK_MAD_TOPS_NOMINAL,
                        "peak_effective_clock_MHz": opcounts.PEAK_CLOCK_MHZ, "peak_source": opcounts.PEAK_SOURCE,
                        "frac": round(x["achieved_Tops_alg"] / opcounts.PEAK_MAD_TOPS, 4),
                        "frac_executed": round(x["achieved_Tops_exec"] / opcounts.PEAK_MAD_TOPS, 4),
                        "frac_vs_nominal_clock": round(x["achieved_Tops_alg"] / opcounts.PEAK_MAD_TOPS_NOMINAL, 4),
                        "traffic": traffic_of(dom),
                        "traffic_source": "profiles/pmc_traffic.json (PMC pass of this build; bytes per step, "
                                          "like achieved)",
                        "algorithmic_work": f"{x['units_per_step']} units x {x['fpmul_per_unit_alg']} Fp-mul x "
                                            f"{opcounts.MAC_PER_FPMUL} MAC per step (executed {x['fpmul_per_unit_exec']} "
                                            f"Fp-mul per unit)",
                        "kernel_ms_alone": x["ms_per_step"],
                        "valu_issue": valu_issue_of(dom, x["ms_per_step"],
                                                    torch.cuda.get_device_properties(dev).multi_processor_count),
                        "timing": "HIP events around each launch on its stream, kernels serialised (one extra "
                                  "slot after the timed region, library timing mode 2)",
                        "slot": {"fpmul_alg_per_step": slot_fpmul, "achieved": round(slot_tops, 3),
                                 "frac": round(slot_tops / opcounts.PEAK_MAD_TOPS, 4),
                                 "note": "all kernels' algorithmic work over ms_per_step (slots in flight overlap)",
                                 **slot_issue(args.workload, elapsed / args.steps,
                                              torch.cuda.get_device_properties(dev).multi_processor_count)},
                        "k_pair3": pair}
        return per, roofline

    # whole-slot effective rate against the r01 (herumi-equivalent, one pairing per partial) work
    verify_effective = world * NP * opcounts.FPMUL_PER_ITEM_R01["verify"] * opcounts.MAC_PER_FPMUL / \
        (elapsed / args.steps) / 1e12

    out = {
        "metric": METRIC, "value": round(value, 1),
        "unit": "items/s (verified partial signatures + ThresholdAggregates)",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        # the ranks' own times (the line takes the slowest) and the RCCL world the library joined
        "per_rank_ms_per_step": [round(x / args.steps * 1e3, 3) for x in per_rank_s],
        "rccl_world": L.hbls_comm_size() if xw else 0,
        **({"rehearsal": f"{world} ranks on ONE GPU, exchange over gloo through host copies: not a measurement"}
           if args.share_device else {}),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u32 (Fp/Fr Montgomery limbs, integer VALU)",
        "data": "synthetic: SHA-256-derived keys, Shamir shares and signing roots (charon_amd/synth.py); "
                "pubshares and signatures produced on device",
        "config": {"workload": wl["desc"], "validators_per_gpu": V, "operators": n, "threshold": t,
                   "aggregated_share_indices": [int(x) + 1 for x in ta_share_positions(n, t)],
                   "distinct_messages": M, "partials_per_gpu": NP, "parallelism": f"validator-sharded x{world}",
                   "slots_in_flight": n_sets, "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                   **({"corrupted_partials_per_gpu": d["n_corrupted"], "bad_frac": bad_frac} if "exp_v" in d else {})},
        "verify_per_s": round(world * NP / (elapsed / args.steps), 1),
        "threshold_aggregate_per_s": round(world * V / (elapsed / args.steps), 1),
        "aggregate_verify_per_s": None if staged else round(world * V / (elapsed / args.steps), 1),
        "mode": args.mode,
        "stage_ms": ({"hash_to_g2": round(k_ms[0], 3), "verify": round(k_ms[1], 3),
                      "threshold_aggregate": round(k_ms[2], 3)} if staged else
                     {"slot": round(k_ms[0], 3), "allgather": round(k_ms[1], 3)}),
        "verify_whole_effective_Tops_vs_r01_work": round(verify_effective, 3),
        "kernels": None,
        "parity": parity, "roofline": None, "cpu_baseline": None,
    }

    if args.host_api and rank == 0 and world == 1:
        st = np.zeros(NP, dtype=np.uint8)
        tout_h = np.zeros(V * 96, dtype=np.uint8)
        tst_h = np.zeros(V, dtype=np.uint8)

        def host_pair():  # charon's flow: parsigex verifies the partials, sigagg aggregates them
            t0 = time.perf_counter()
            _chk(L, L.hbls_verify_batch(_p(d["pks"]), _p(d["sigs"]), _p(d["item_msgs"]), _p(d["item_off"]),
                                        _p(d["item_len"]), NP, _p(st)))
            t1 = time.perf_counter()
            _chk(L, L.hbls_threshold_aggregate_batch(_p(d["ta_sigs"]), _p(d["ta_idx"]), _p(d["grp_off"]), V,
                                                     _p(tout_h), _p(tst_h)))
            t2 = time.perf_counter()
            return t2 - t0, t1 - t0, t2 - t1

        host_pair()  # warm-up: staging buffers and workspaces grow once
        runs = [host_pair() for _ in range(args.host_runs)]
        med = sorted(runs)[len(runs) // 2]
        out["host_buffer_items_per_s"] = round((NP + V) / med[0], 1)
        out["host_buffer_runs_ms"] = [[round(x * 1e3, 2) for x in r] for r in runs]  # (pair, verify, aggregate)
        # the same with every key (pubshares and DV keys) in the library's key cache, as charon
        # loads its cluster lock at startup (hbls_pubkey_cache_add); the cache is emptied after
        _chk(L, L.hbls_pubkey_cache_add(_p(d["pks"]), NP))
        kruns = [host_pair() for _ in range(args.host_runs)]
        _chk(L, L.hbls_pubkey_cache_clear())
        out["host_buffer_items_per_s_key_cache"] = round((NP + V) / sorted(kruns)[len(kruns) // 2][0], 1)
        if "exp_v" in d:
            clean = d["exp_agg"] == 0  # members all valid: the aggregate is the root signature
            out["host_buffer_parity"] = bool(np.array_equal(st, d["exp_v"]) and np.array_equal(tst_h, d["exp_ta"]) and
                                             np.array_equal(tout_h.reshape(V, 96)[clean],
                                                            d["root_sigs"].reshape(V, 96)[clean]))
        else:
            out["host_buffer_parity"] = bool((st == 0).all() and (tst_h == 0).all() and
                                             np.array_equal(tout_h, d["root_sigs"]))
        # the rate the Go shim sees (host buffers, PCIe both ways, partial Verify then
        # ThresholdAggregate as two calls); never the headline
        out["pcie_inclusive_items_per_s"] = out["host_buffer_items_per_s"]
        # the same pair of calls from several threads at once (charon's goroutines: parsigex and
        # sigagg of different duties); each call owns a host-call context, so their transfers and
        # kernels overlap on the device (hipbls.hip Hc)
        if args.host_threads > 1:
            rounds = 2
            res = [None] * args.host_threads

            def worker(k):
                st_k = np.zeros(NP, dtype=np.uint8)
                to_k = np.zeros(V * 96, dtype=np.uint8)
                ts_k = np.zeros(V, dtype=np.uint8)
                ok = True
                for _ in range(rounds):
                    rc1 = L.hbls_verify_batch(_p(d["pks"]), _p(d["sigs"]), _p(d["item_msgs"]), _p(d["item_off"]),
                                              _p(d["item_len"]), NP, _p(st_k))
                    rc2 = L.hbls_threshold_aggregate_batch(_p(d["ta_sigs"]), _p(d["ta_idx"]), _p(d["grp_off"]), V,
                                                           _p(to_k), _p(ts_k))
                    ok = ok and rc1 == 0 and rc2 == 0 and np.array_equal(st_k, st) and np.array_equal(ts_k, tst_h) \
                        and np.array_equal(to_k, tout_h)
                res[k] = ok

            ths = [threading.Thread(target=worker, args=(k,)) for k in range(args.host_threads)]
            t0 = time.perf_counter()
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            dt = time.perf_counter() - t0
            out["host_buffer_concurrent"] = {
                "threads": args.host_threads, "calls_per_thread": 2 * rounds,
                "items_per_s": round(args.host_threads * rounds * (NP + V) / dt, 1),
                "same_results_as_sequential": all(res)}

    if rank == 0 and world == 1 and args.key_tables and not staged:
        out["with_key_tables"] = key_table_slots(L, d_pk, d_dvpk, outs, NP, V, args.steps, step_slot, mk, items)

    if os.environ.get("HBLS_STATS") == "1":  # fallback counters over the whole run (diagnosis)
        st = (ctypes.c_uint64 * 6)()
        _chk(L, L.hbls_stats(st, 6))
        out["fallback_stats"] = dict(zip(("items", "groups", "fallback_items", "last_chunk_groups_checked",
                                          "slot_checks", "slot_checks_failed"), list(st)))
    out["kernels"], out["roofline"] = kernel_roofline()

    if rank == 0 and world == 1 and "exp_v" in d and not staged:
        out["first_error"] = first_error_verify(L, d, d_pk, d_sig, d_midx, d_vgoff, dev, sp)
        parity["first_error_index_exact"] = out["first_error"]["first_index_exact"]

    if rank == 0 and world == 1 and args.aggregate_verify:
        out["verify_aggregate"] = aggregate_verify(L, d, d_pk, dev, sp)
        parity["verify_aggregate_ok"] = all(x["all_ok"] for x in out["verify_aggregate"].values())

    if rank == 0 and world == 1 and args.callers > 0:
        out["concurrent_callers"] = concurrent_callers(L, d, args.callers, args.callers_seconds)
        # one unchanged tbls.Verify caller (parsigex.go:94 verifies serially per stream) on an idle library
        out["single_call_latency_ms"] = out["concurrent_callers"]["single_call_latency_ms"]

    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(d, args.cpu_seconds)

    if xw:
        if L.hbls_comm_size() != world and not args.share_device:
            parity["rccl_world_matches"] = False
        _chk(L, L.hbls_comm_destroy())
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if not all(parity.values()):
        print("PARITY FAILURE: " + json.dumps(parity), file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
