#!/usr/bin/env python3
"""bench.py -- charon's BLS hot path on MI355X (BASELINE.json metric).

One step = one attestation slot of BASELINE.json configs[1] ("C2"): for V = 10 000 validators of a
4-operator threshold-3 cluster,
  1. hash the slot's 64 distinct signing roots to G2          (k_hash_to_g2)
  2. verify all V*n = 40 000 partial signatures                (k_verify: tbls.Verify,
     /root/reference/tbls/herumi.go:288-304, callers core/parsigex/parsigex.go:93-98)
  3. threshold-aggregate every validator's first t partials   (k_group_member + k_group_sum:
     tbls.ThresholdAggregate, herumi.go:249-286, caller core/sigagg/sigagg.go:105).
Inputs (compressed pubshares, partial signatures, messages, share indices) are resident in HBM
before the timed region; outputs are per-item status bytes and 96-byte aggregates in HBM.

value = (verified partials + threshold aggregates) per second summed over all ranks.  Weak
scaling: every rank owns its own V validators (validator sharding); with N > 1
ranks each step ends with the RCCL all-gather of verdicts and aggregates over xGMI.

roofline: integer VALU: k_verify's algorithmic 32-bit multiply-adds per launch
divided by its HIP-event duration, against the measured v_mad_u64_u32 peak.
cpu_baseline: the same per-item arithmetic compiled for the host by g++ (tests/native/hostcheck.cpp,
a port -- herumi and the Go toolchain are absent), timed on a bounded sample of validators.
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from charon_amd.opcounts import FPMUL_PER_ITEM, MAC_PER_FPMUL, PEAK_MAD_TOPS  # noqa: E402
from charon_amd.shard import SlotExchange, max_over_ranks, owned_validators  # noqa: E402

N_LINES = 68  # Miller-loop lines per pairing (pairing.h)

METRIC = "verified partial sigs/sec + ThresholdAggregate/sec per node, 1-8 MI355X"

WORKLOADS = {
    "c2": dict(validators=10_000, n=4, t=3, distinct=False, n_msgs=64,
               desc="C2 (BASELINE configs[1]): 10k validators, 4-operator threshold-3 cluster, one attestation "
                    "slot with 64 committee signing roots: 40k partial Verify + 10k ThresholdAggregate"),
    "c3": dict(validators=100_000, n=10, t=7, distinct=True, n_msgs=0,
               desc="C3 (BASELINE configs[2]): 100k validators, 10-operator threshold-7 cluster, distinct "
                    "per-validator messages: 1M partial Verify + 100k ThresholdAggregate"),
}


def _p(x) -> ctypes.c_void_p:
    """Device pointer of a torch tensor or host pointer of a numpy array."""
    if isinstance(x, np.ndarray):
        return ctypes.c_void_p(x.ctypes.data)
    return ctypes.c_void_p(x.data_ptr())


def _chk(L, rc):
    if rc != 0:
        raise RuntimeError("hipbls: " + L.hbls_last_error().decode(errors="replace"))


def setup_inputs(L, wl, V, rank):
    """Synthetic cluster -> host arrays; keys and signatures are derived on the GPU."""
    from charon_amd import synth
    n, t = wl["n"], wl["t"]
    cl = synth.make_cluster(V, n, t, first_validator=owned_validators(rank, V).start, n_msgs=wl["n_msgs"] or 64,
                            distinct_messages=wl["distinct"])
    NP = V * n
    M = len(cl.msgs)
    msg_of_v = np.asarray(cl.msg_of_validator, dtype=np.uint32)
    midx = np.repeat(msg_of_v, n)
    msgs = np.frombuffer(b"".join(cl.msgs), dtype=np.uint8).copy()
    moff = (np.arange(M, dtype=np.uint64) * 32)
    mlen = np.full(M, 32, dtype=np.uint32)
    # per-item message tables for the host-buffer sign calls
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
    stv = np.zeros(V, dtype=np.uint8)
    root_off = np.arange(V, dtype=np.uint64) * 32  # named: a temporary would be freed before the call
    root_len = np.full(V, 32, dtype=np.uint32)
    _chk(L, L.hbls_sign_batch(_p(root_sks), _p(root_msgs), _p(root_off), _p(root_len), V, _p(root_sigs),
                              _p(stv)))
    assert not stv.any(), "root signing failed"
    # ThresholdAggregate input: shares 1..t of every validator (parsigdb fires with exactly t,
    # core/parsigdb/memory.go:218-221)
    sel = (np.arange(V)[:, None] * n + np.arange(t)[None, :]).reshape(-1)
    ta_sigs = sigs.reshape(NP, 96)[sel].reshape(-1).copy()
    ta_idx = np.tile(np.arange(1, t + 1, dtype=np.int64), V)
    grp_off = (np.arange(V + 1, dtype=np.uint32) * t)
    return dict(n=n, t=t, V=V, NP=NP, M=M, msgs=msgs, moff=moff, mlen=mlen, midx=midx, pks=pks, sigs=sigs,
                item_msgs=item_msgs, item_off=item_off, item_len=item_len, ta_sigs=ta_sigs, ta_idx=ta_idx,
                grp_off=grp_off, root_sigs=root_sigs)


def cpu_baseline(d, seconds: float):
    """The host restatement (g++ build of the kernels' per-item arithmetic) on a bounded sample.

    One unit = one validator: n partial Verifies (each hashing its message, as herumi's VerifyByte
    does) + one ThresholdAggregate over t partials, checked against the root-key signature.  The
    loop is native (tests/native/hostcheck.cpp hc_cpu_slot, std::thread workers); threads = usable
    host cores, at most 16."""
    from charon_amd.build import build_hostcheck
    hc = ctypes.CDLL(build_hostcheck(verbose=False))
    n, t = d["n"], d["t"]
    midx = np.ascontiguousarray(d["midx"], dtype=np.uint32)
    try:
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        threads = max(1, min(16, os.cpu_count() or 1))

    def run(units, th):
        t0 = time.perf_counter()
        bad = hc.hc_cpu_slot(th, units, n, t, _p(d["pks"]), _p(d["sigs"]), _p(d["msgs"]), _p(midx),
                             _p(d["ta_sigs"]), _p(d["root_sigs"]))
        return time.perf_counter() - t0, bad

    per_unit, bad = run(1, 1)
    units = int(min(d["V"], max(threads, seconds * threads / max(per_unit, 1e-6))))
    wall, bad2 = run(units, threads)
    return {"value": round(units * (n + 1) / wall, 2),
            "unit": "items/s (verified partial signatures + ThresholdAggregates)",
            "cores": threads, "kind": "port",
            "sample": f"{units} validators x ({n} partial Verify + 1 ThresholdAggregate of {t}) of the same "
                      f"synthetic cluster; g++ -O2 build of the kernels' per-item arithmetic "
                      f"(tests/native/hostcheck.cpp hc_cpu_slot, {threads} std::threads), one hash_to_G2 per "
                      f"Verify as herumi does; not herumi (absent offline)",
            "agrees_with_expected": bad == 0 and bad2 == 0, "wall_s": round(wall, 2)}


def main(argv=None):
    ap = argparse.ArgumentParser(description="charon BLS hot path on MI355X")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--validators", type=int, default=0, help="override validators per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample (0: skip)")
    ap.add_argument("--host-api", action="store_true", help="also time the host-buffer (PCIe-inclusive) entry points")
    ap.add_argument("--mode", default="slot", choices=["slot", "staged"],
                    help="slot: one hbls_slot_device call per step (stages overlap); staged: stage by stage")
    args = ap.parse_args(argv)

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus and rank == 0:
        print(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from charon_amd import _lib
    L = _lib.load_library()
    _chk(L, L.hbls_init(local))

    wl = WORKLOADS[args.workload]
    V = args.validators or wl["validators"]
    d = setup_inputs(L, wl, V, rank)
    n, t, NP, M = d["n"], d["t"], d["NP"], d["M"]
    dev = torch.device("cuda", local)

    def up(a):
        return torch.from_numpy(a).to(dev)

    d_msg, d_moff, d_mlen = up(d["msgs"]), up(d["moff"].view(np.int64)), up(d["mlen"].view(np.int32))
    d_midx, d_pk, d_sig = up(d["midx"].view(np.int32)), up(d["pks"]), up(d["sigs"])
    d_tsig, d_tidx, d_goff = up(d["ta_sigs"]), up(d["ta_idx"]), up(d["grp_off"].view(np.int32))
    d_hm = torch.zeros(M * L.hbls_hm_entry_bytes(), dtype=torch.uint8, device=dev)
    d_vst = torch.full((NP,), 255, dtype=torch.uint8, device=dev)
    d_tout = torch.zeros(V * 96, dtype=torch.uint8, device=dev)
    d_tst = torch.full((V,), 255, dtype=torch.uint8, device=dev)
    xchg = SlotExchange(world, V, d["n"], dev) if world > 1 else None

    stream = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(stream.cuda_stream)

    def step_slot(ev):
        # the slot entry point: hashing, verification and threshold aggregation overlap on the
        # library's side streams; ordered on `stream`
        ev[0].record(stream)
        _chk(L, L.hbls_slot_device(_p(d_msg), _p(d_moff), _p(d_mlen), M, _p(d_hm), _p(d_pk), _p(d_sig), _p(d_midx),
                                   NP, _p(d_vst), _p(d_tsig), _p(d_tidx), _p(d_goff), V, V * t, _p(d_tout),
                                   _p(d_tst), sp))
        ev[1].record(stream)
        if world > 1:  # all-gather verdicts + compressed aggregates to every rank
            with torch.cuda.stream(stream):
                xchg.exchange(d_vst, d_tout, d_tst)
        ev[2].record(stream)

    def step_staged(ev):
        # the same work stage by stage (no overlap): per-stage event timings
        ev[0].record(stream)
        _chk(L, L.hbls_hash_to_g2_device(_p(d_msg), _p(d_moff), _p(d_mlen), M, _p(d_hm), sp))
        ev[1].record(stream)
        _chk(L, L.hbls_verify_device(_p(d_pk), _p(d_sig), _p(d_midx), _p(d_hm), NP, _p(d_vst), sp))
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
    _chk(L, L.hbls_timing(1))
    evs = [mk() for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, dev)

    seg = np.array([[e[i].elapsed_time(e[i + 1]) for i in range(n_ev - 1)] for e in evs])  # ms
    k_ms = seg.mean(axis=0)
    # k_pair3 (the dominant kernel) durations: HIP events the library records on its stream
    pm = (ctypes.c_float * 4096)()
    npm = ctypes.c_size_t(0)
    _chk(L, L.hbls_timing_read(pm, 4096, ctypes.byref(npm)))
    _chk(L, L.hbls_timing(0))
    pair3_ms = float(np.sum(np.frombuffer(pm, dtype=np.float32, count=npm.value))) / args.steps

    # parity of the timed outputs: every partial verifies, every aggregate is byte-identical to the
    # root-key signature (tbls_test.go:72-97 property), every status OK
    vst = d_vst.cpu().numpy()
    tst = d_tst.cpu().numpy()
    tout = d_tout.cpu().numpy()
    parity = {"verify_all_ok": bool((vst == 0).all()), "ta_all_ok": bool((tst == 0).all()),
              "ta_equals_root_signature": bool(np.array_equal(tout, d["root_sigs"]))}
    if world > 1:
        parity["allgather_ok"] = xchg.all_ok()

    items = world * (NP + V)
    ms_per_step = elapsed / args.steps * 1e3
    value = items / (elapsed / args.steps)

    fpmul_pair = FPMUL_PER_ITEM["k_pair3"]
    t_pair = pair3_ms * 1e-3
    pair_bytes = NP * (112 + 1 + 1 + 1 + 4 + 2 * N_LINES * 288 + 1)  # P, 3 status bytes, msg index, 2x68 lines, out
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f).get(args.workload, {}).get("k_pair3")
        if pmc and pmc.get("partials") == NP:
            traffic = pmc["hbm_bytes_per_launch"]
    achieved = NP * fpmul_pair * MAC_PER_FPMUL / t_pair / 1e12 if t_pair > 0 else None
    roofline = {"bound": "valu", "kernel": "k_pair3", "achieved": achieved and round(achieved, 3),
                "peak": PEAK_MAD_TOPS, "unit": "Tops/s (32-bit multiply-add lane-ops, v_mad_u64_u32)",
                "frac": achieved and round(achieved / PEAK_MAD_TOPS, 4), "traffic": traffic,
                "kernel_ms": round(pair3_ms, 3),
                "algorithmic_work": f"{fpmul_pair} Fp-mul x {MAC_PER_FPMUL} MAC per partial x {NP} partials "
                                    f"(2-pair Miller loop + final exponentiation, frozen r01 count)",
                "algorithmic_bytes_per_launch": pair_bytes,
                "hbm_GBps_algorithmic": round(pair_bytes / t_pair / 1e9, 3) if t_pair > 0 else None}
    # whole Verify (decompression + lines + pairing) per partial, frozen r01 count, over the step
    verify_effective = world * NP * FPMUL_PER_ITEM["k_verify"] * MAC_PER_FPMUL / (elapsed / args.steps) / 1e12

    out = {
        "metric": METRIC, "value": round(value, 1),
        "unit": "items/s (verified partial signatures + ThresholdAggregates)",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u32 (Fp/Fr Montgomery limbs, integer VALU)",
        "data": "synthetic: SHA-256-derived keys, Shamir shares and signing roots (charon_amd/synth.py); "
                "pubshares and signatures produced on device",
        "config": {"workload": wl["desc"], "validators_per_gpu": V, "operators": n, "threshold": t,
                   "distinct_messages": M, "partials_per_gpu": NP, "parallelism": f"validator-sharded x{world}"},
        "verify_per_s": round(world * NP / (elapsed / args.steps), 1),
        "threshold_aggregate_per_s": round(world * V / (elapsed / args.steps), 1),
        "mode": args.mode,
        "stage_ms": ({"hash_to_g2": round(k_ms[0], 3), "verify": round(k_ms[1], 3),
                      "threshold_aggregate": round(k_ms[2], 3)} if staged else
                     {"slot": round(k_ms[0], 3), "allgather": round(k_ms[1], 3)}),
        "verify_whole_effective_Tops": round(verify_effective, 3),
        "parity": parity, "roofline": roofline, "cpu_baseline": None,
    }

    if args.host_api and rank == 0:
        st = np.zeros(NP, dtype=np.uint8)
        t0 = time.perf_counter()
        _chk(L, L.hbls_verify_batch(_p(d["pks"]), _p(d["sigs"]), _p(d["item_msgs"]), _p(d["item_off"]),
                                    _p(d["item_len"]), NP, _p(st)))
        tout_h = np.zeros(V * 96, dtype=np.uint8)
        tst_h = np.zeros(V, dtype=np.uint8)
        _chk(L, L.hbls_threshold_aggregate_batch(_p(d["ta_sigs"]), _p(d["ta_idx"]), _p(d["grp_off"]), V,
                                                 _p(tout_h), _p(tst_h)))
        out["host_buffer_items_per_s"] = round((NP + V) / (time.perf_counter() - t0), 1)

    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(d, args.cpu_seconds)

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
