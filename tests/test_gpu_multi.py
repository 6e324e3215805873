"""The library's own multi-GPU code on the one-GPU box (-m gpu), through the C ABI.

* RCCL exchange: the library's communicator (hbls_comm_unique_id / hbls_comm_init) as a world of
  one on the GPU, driven by bench.py's own exchange code (charon_amd/shard.py SlotExchange with
  library_allgather on one exchange stream, two output sets in flight): the gathered bytes are the
  rank's own.  (Two ranks cannot share one GPU under RCCL; the N-rank ordering is covered over gloo
  by tests/test_shard.py, the same class.)
* In-process device split (charon is one Go process over every GPU of the node, app/app.go:131):
  hbls_debug_split drives the device through two and three contexts, so every host-buffer entry
  point shards its items over them with one host thread each (hipbls.hip for_each_device), exactly
  as over several GPUs.  Verdicts, aggregates, signatures, keys and roots equal the unsplit run.
* The public-key cache under concurrency: adds racing verifications on other threads (lock order
  of hbls_pubkey_cache_add vs. a verification's device lock), verdicts unchanged.
* Soundness of the per-group check without the batched final exponentiation: a group of ONE
  partial with a folded aggregate, errors +D on the partial and -D on the aggregate, must reject
  both (core/sigagg/sigagg.go:117 folded into the partial's group).
"""
import ctypes
import os
import hashlib
import random
import threading

import numpy as np
import pytest

from charon_amd import _lib
from charon_amd._lib import BAD_PUBKEY, NOT_VERIFIED, OK

pytestmark = pytest.mark.gpu


def _p(x):
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        return ctypes.c_void_p(x.ctypes.data)
    return ctypes.c_void_p(x.data_ptr())


@pytest.fixture(scope="module")
def L(hipbls):
    return _lib.load_library()


def test_rccl_world_of_one_slot_exchange(L):
    import torch
    from charon_amd.shard import SlotExchange, init_library_comm, library_allgather
    dev = torch.device("cuda", 0)
    V, n = 1000, 7
    torch.zeros(1, device=dev)  # torch's HIP context first, as bench.py does (torch.cuda.set_device)
    init_library_comm(L, 1, 0)
    try:
        exch = SlotExchange(1, 0, {"vst": V * n, "tout": V * 96, "tst": V, "ast": V}, dev, library_allgather(L),
                            stream=torch.cuda.Stream(device=dev))
        sets = [exch.gather_buffers() for _ in range(2)]
        producers = [torch.cuda.Stream(device=dev) for _ in range(2)]
        g = torch.Generator().manual_seed(5)
        sent = []
        for slot in range(4):
            k = slot % 2
            outs = {f: torch.randint(0, 256, (m,), dtype=torch.uint8, generator=g) for f, m in exch.sizes.items()}
            with torch.cuda.stream(producers[k]):
                outs = {f: t.to(dev, non_blocking=False) for f, t in outs.items()}
            assert exch.exchange(outs, sets[k], producer=producers[k]) == slot
            sent.append((k, {f: t.cpu() for f, t in outs.items()}))
            producers[k].synchronize()
            for f in exch.sizes:
                assert torch.equal(sets[k][f].cpu(), sent[-1][1][f]), (slot, f)
        assert exch.issued == [(s, f) for s in range(4) for f in ("vst", "tout", "tst", "ast")]
        # the communicator is one per process and one device per process
        assert L.hbls_comm_init(1, 0, _p(np.zeros(L.hbls_comm_id_bytes(), dtype=np.uint8))) == 0  # idempotent
    finally:
        assert L.hbls_comm_destroy() == 0
    assert L.hbls_allgather_device(None, None, 0, None) != 0  # no communicator any more
    assert b"no communicator" in L.hbls_last_error()


def test_status_bitmap(L):
    """hbls_status_bitmap (the verify bitmap the ranks all-gather): bit i of byte i / 8, least
    significant first, set for HBLS_OK -- against numpy's packbits, on lengths around the wave
    (64 statuses per ballot) and byte boundaries"""
    import torch
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    rng = np.random.default_rng(9)
    for n in (1, 7, 8, 63, 64, 65, 1000, 4099):
        st = rng.integers(0, 4, n, dtype=np.uint8)
        st[rng.random(n) < 0.5] = OK
        d_st = torch.from_numpy(st).to(dev)
        bits = torch.full(((n + 7) // 8,), 0xA5, dtype=torch.uint8, device=dev)
        assert L.hbls_status_bitmap(_p(d_st), n, _p(bits), ctypes.c_void_p(s.cuda_stream)) == 0
        s.synchronize()
        assert np.array_equal(bits.cpu().numpy(), np.packbits(st == OK, bitorder="little")), n


def _mixed_inputs(hipbls, rng, n_keys=48, n_items=700):
    keys = [hipbls.generate_secret_key() for _ in range(n_keys)]
    pks = [hipbls.secret_to_public_key(k) for k in keys]
    msgs = [hashlib.sha256(b"split duty %d" % (i % 9)).digest() for i in range(n_keys)]
    sigs = hipbls.sign_batch(keys, msgs)
    items = []
    for i in range(n_items):
        j = rng.randrange(n_keys)
        c = rng.random()
        if c < 0.05:
            items.append((pks[j], hashlib.sha256(b"wrong").digest(), sigs[j]))
        elif c < 0.08:
            items.append((pks[(j + 1) % n_keys], msgs[j], sigs[j]))
        elif c < 0.10:
            items.append((bytes([0x9A]) + b"\xff" * 47, msgs[j], sigs[j]))
        elif c < 0.12:
            items.append((pks[j], msgs[j], bytes([0xC0]) + bytes(95)))
        else:
            items.append((pks[j], msgs[j], sigs[j]))
    return keys, pks, msgs, sigs, items


def _everything(hipbls, keys, pks, msgs, sigs, items, rng_seed):
    """Every host-buffer entry point once, on fixed inputs."""
    rng = random.Random(rng_seed)
    P, M, S = zip(*items)
    out = {"verify": hipbls.verify_batch(P, M, S)}
    groups = []
    for g in range(37):
        ids = sorted(rng.sample(range(1, 8), rng.choice([1, 3, 5])))
        groups.append({i: sigs[(g + i) % len(sigs)] for i in ids})
    groups[5] = {}
    out["ta"] = hipbls.threshold_aggregate_batch(groups)
    out["agg"] = hipbls.aggregate_batch([sigs[g:g + 1 + g % 5] for g in range(30)] + [[]])
    vgroups = [pks[g:g + 1 + g % 7] for g in range(20)]
    out["va"] = hipbls.verify_aggregate_batch(vgroups, [out["agg"][0][g] for g in range(20)], [msgs[g] for g in range(20)])
    out["sign"] = hipbls.sign_batch(keys, [msgs[(i + 3) % len(msgs)] for i in range(len(keys))])
    out["pk"] = [hipbls.secret_to_public_key(k) for k in keys[:5]]
    from charon_amd import signing_roots
    doms = [hashlib.sha256(b"domain %d" % k).digest() for k in range(3)]
    out["roots"] = signing_roots.signing_roots(msgs * 3, doms, [k % 3 for k in range(3 * len(msgs))])
    return out


def test_debug_split_same_results(L, hipbls):
    rng = random.Random(11)
    keys, pks, msgs, sigs, items = _mixed_inputs(hipbls, rng)
    base = _everything(hipbls, keys, pks, msgs, sigs, items, 3)
    # the verdicts are the per-item ones (the construction's)
    assert base["verify"].count(OK) < len(items) and BAD_PUBKEY in base["verify"] and NOT_VERIFIED in base["verify"]
    try:
        for copies in (2, 3):
            assert L.hbls_debug_split(copies) == 0
            assert L.hbls_device_count() == copies
            got = _everything(hipbls, keys, pks, msgs, sigs, items, 3)
            assert got == base, copies
            # the key cache follows the split: every context holds the cached keys
            hipbls.clear_pubkey_cache()
            hipbls.cache_pubkeys(pks[:30])
            P, M, S = zip(*items)
            assert hipbls.verify_batch(P, M, S) == base["verify"]
            hipbls.clear_pubkey_cache()
    finally:
        assert L.hbls_debug_split(1) == 0
    assert L.hbls_device_count() == 1
    assert L.hbls_debug_split(0) != 0


def test_cache_add_races_verification(hipbls):
    """hbls_pubkey_cache_add and _clear on one thread while four threads verify: no deadlock (the
    add takes the device locks one at a time and the key map last), every verdict right.  After each
    clear the next add reuses table indices 0.. for OTHER keys, so a lookup made outside the device
    lock, or a table rewritten under a verification still in flight, would check a signature against
    the wrong key (hipbls.hip kc_lookup / kc_fill)."""
    rng = random.Random(21)
    keys, pks, msgs, sigs, items = _mixed_inputs(hipbls, rng, n_keys=64, n_items=200)
    P, M, S = zip(*items)
    want = hipbls.verify_batch(P, M, S)
    errs = []
    stop = threading.Event()

    def verifier(w):
        try:
            while not stop.is_set():
                lo = (w * 37) % 150
                got = hipbls.verify_batch(P[lo:lo + 50], M[lo:lo + 50], S[lo:lo + 50])
                if got != want[lo:lo + 50]:
                    errs.append((w, lo))
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    def adder():
        try:
            for r in range(24):
                hipbls.cache_pubkeys(pks[(r * 5) % 64:(r * 5) % 64 + 8])
                if r % 3 == 2:
                    hipbls.clear_pubkey_cache()
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=verifier, args=(w,)) for w in range(4)]
    ad = threading.Thread(target=adder)
    for t in th:
        t.start()
    ad.start()
    ad.join(timeout=60)
    stop.set()
    for t in th:
        t.join(timeout=60)
    assert not ad.is_alive() and not any(t.is_alive() for t in th), "deadlock"
    hipbls.clear_pubkey_cache()
    assert not errs, errs[:5]


def test_singleton_group_folded_aggregate_cancelling_errors(L, hipbls):
    """Groups of ONE partial, each with its folded post-aggregate verification (hbls_slot_device,
    dv_pks set), below the batched final exponentiation's threshold (per-group checks): group 1's
    partial carries +D and its aggregate -D.  Both must be rejected; the other groups pass."""
    import torch
    from oracle import bls12381 as B
    prev = L.hbls_fe_batch(0)
    try:
        G = 4
        m = hashlib.sha256(b"singleton").digest()
        sks = [hipbls.generate_secret_key() for _ in range(G)]
        dvsks = [hipbls.generate_secret_key() for _ in range(G)]
        pks = [hipbls.secret_to_public_key(k) for k in sks]
        dvpks = [hipbls.secret_to_public_key(k) for k in dvsks]
        sigs = hipbls.sign_batch(sks, [m] * G)
        dvsigs = hipbls.sign_batch(dvsks, [m] * G)
        D = B.g2_decompress(hipbls.sign(hipbls.generate_secret_key(), m))
        sigs[1] = B.g2_compress(B.g2_add(B.g2_decompress(sigs[1]), D))
        dvsigs[1] = B.g2_compress(B.g2_add(B.g2_decompress(dvsigs[1]), B.g2_neg(D)))
        dev = torch.device("cuda", 0)
        up = lambda a: torch.from_numpy(np.frombuffer(a, dtype=np.uint8).copy()).to(dev)  # noqa: E731
        dm, dpk, dsig, ddv, dts = up(m), up(b"".join(pks)), up(b"".join(sigs)), up(b"".join(dvpks)), up(b"".join(dvsigs))
        moff = torch.zeros(1, dtype=torch.int64, device=dev)
        mlen = torch.full((1,), 32, dtype=torch.int32, device=dev)
        midx = torch.zeros(G, dtype=torch.int32, device=dev)
        goff = torch.arange(G + 1, dtype=torch.int32, device=dev)
        tidx = torch.ones(G, dtype=torch.int64, device=dev)  # k = 1: the aggregate is the member itself
        hm = torch.zeros(L.hbls_hm_entry_bytes(), dtype=torch.uint8, device=dev)
        vst = torch.full((G,), 255, dtype=torch.uint8, device=dev)
        tout = torch.zeros(G * 96, dtype=torch.uint8, device=dev)
        tst = torch.full((G,), 255, dtype=torch.uint8, device=dev)
        ast = torch.full((G,), 255, dtype=torch.uint8, device=dev)
        slot = _lib.HblsSlot(msgs=_p(dm).value, msg_off=_p(moff).value, msg_len=_p(mlen).value, n_msgs=1, hm=_p(hm).value,
                             pks=_p(dpk).value, sigs=_p(dsig).value, msg_idx=_p(midx).value, n=G, vgrp_off=_p(goff).value,
                             n_vgroups=G, vstatus=_p(vst).value, ta_sigs=_p(dts).value, ta_src=None, ta_idx=_p(tidx).value,
                             grp_off=_p(goff).value, n_groups=G, n_ta_partials=G, ta_out=_p(tout).value,
                             ta_status=_p(tst).value, dv_pks=_p(ddv).value, agg_vstatus=_p(ast).value)
        s = torch.cuda.Stream(device=dev)
        assert L.hbls_slot_device(ctypes.byref(slot), ctypes.c_void_p(s.cuda_stream)) == 0, L.hbls_last_error()
        s.synchronize()
        assert list(vst.cpu().numpy()) == [OK, NOT_VERIFIED, OK, OK]
        assert list(tst.cpu().numpy()) == [OK] * G
        assert list(ast.cpu().numpy()) == [OK, NOT_VERIFIED, OK, OK]
        assert bytes(tout.cpu().numpy()[:96]) == dvsigs[0]
    finally:
        L.hbls_fe_batch(prev)


@pytest.mark.parametrize("workload", ["c5", "c3"])
def test_bench_two_ranks_rehearsal(workload):
    """bench.py's N > 1 path end to end on the one-GPU box: `--gpus 2` starts two ranks itself
    (launch_ranks), both on device 0 (`--share-device 1`; RCCL refuses two ranks on one GPU, so the
    slot exchange runs over gloo through host copies -- the library's RCCL all-gather is covered as
    a world of one above).  Every rank builds its own shard, runs its slots, exchanges the packed
    verdicts and aggregates every slot, checks every rank's gathered blocks (C5: its own block
    against its construction; C3: every rank's block all valid, its own aggregates equal to the
    root signatures), and rank 0 prints one line with n_gpus 2 and both ranks' times."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--share-device", "1", "--workload", workload,
           "--validators", "3000" if workload == "c5" else "2000", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0",
           "--callers", "0", "--aggregate-verify", "0", "--key-tables", "0", "--host-api", "0"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280)
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, (p.returncode, p.stdout[-1500:], p.stderr[-3000:])
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and "rehearsal" in line and len(line["per_rank_ms_per_step"]) == 2
    assert line["parity"] and all(line["parity"].values()), line["parity"]
    assert "allgather_ok" in line["parity"]
