"""N > 1 path on CPU: validator sharding and the slot's all-gather (charon_amd/shard.py, bench.py
--gpus N) with world_size 2 over gloo.

The sharded cluster must be the unsharded one split in rank order (weak scaling: rank r owns
validators [r*V, (r+1)*V)), and after the exchange every rank must hold every rank's verdicts,
aggregates and statuses in global validator order.  The exchange is bench.py's own code
(shard.SlotExchange, with gloo in place of the library's RCCL all-gather): several slots in flight
over two output sets, every rank issuing its collectives in the same (slot, field) order.  The
per-rank slot results are stand-ins (deterministic bytes derived from each validator's shares and
the slot number); the GPU computes the real ones.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from charon_amd import synth
from charon_amd.shard import (FIELDS, PACK_FIELDS, SlotExchange, gloo_allgather, max_over_ranks, owned_validators,
                               pack_layout, pack_views, unpack_gathered)

V, N, T, WORLD = 3, 4, 3, 2


def _slot_results(cl, slot=0):
    """Stand-in slot outputs of one shard: verdict byte per partial, 96 B, an aggregation status and
    a post-aggregate verification status per validator."""
    vst = torch.tensor([(sk[0] + slot) % 5 for sk in cl.share_sks], dtype=torch.uint8)
    tout = torch.tensor([(b + slot) % 256 for b in b"".join(r * 3 for r in cl.root_sks)], dtype=torch.uint8)
    tst = torch.tensor([(r[-1] + slot) % 3 for r in cl.root_sks], dtype=torch.uint8)
    ast = torch.tensor([(r[-2] + slot) % 4 for r in cl.root_sks], dtype=torch.uint8)
    # the verify bitmap bench.py exchanges (hbls_status_bitmap: bit i set for status 0)
    vbits = torch.from_numpy(np.packbits(vst.numpy() == 0, bitorder="little"))
    return {"vst": vst, "vbits": vbits, "tout": tout, "tst": tst, "ast": ast}


def _worker(rank, port, errq):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        first = owned_validators(rank, V).start
        cl = synth.make_cluster(V, N, T, first_validator=first)
        full = synth.make_cluster(WORLD * V, N, T)
        # sharding == the unsharded cluster split in rank order
        assert cl.root_sks == full.root_sks[first:first + V]
        assert cl.share_sks == full.share_sks[first * N:(first + V) * N]
        assert [cl.msgs[m] for m in cl.msg_of_validator] == [full.msgs[m] for m in full.msg_of_validator][first:first + V]
        shards = [synth.make_cluster(V, N, T, first_validator=owned_validators(r, V).start) for r in range(WORLD)]
        exch = SlotExchange(WORLD, rank, {"vst": V * N, "vbits": (V * N + 7) // 8, "tout": V * 96, "tst": V, "ast": V},
                            "cpu", gloo_allgather)
        sets = [exch.gather_buffers() for _ in range(2)]  # two slots in flight, as bench.py --inflight 2
        for slot in range(5):
            recv = sets[slot % 2]
            assert exch.exchange(_slot_results(cl, slot), recv) == slot
            want = {f: torch.cat([_slot_results(sh, slot)[f] for sh in shards]) for f in exch.sizes}
            for f in exch.sizes:
                assert torch.equal(recv[f], want[f]), (slot, f)
                for r in range(WORLD):
                    assert torch.equal(exch.block(recv, f, r), _slot_results(shards[r], slot)[f])
            # global validator order: the unsharded cluster's aggregates
            assert torch.equal(recv["tout"], _slot_results(full, slot)["tout"])
        # every rank issued the same collectives in the same order
        logs = [None] * WORLD
        dist.all_gather_object(logs, exch.issued)
        assert logs[0] == logs[1] == [(k, f) for k in range(5) for f in exch.sizes], logs
        assert set(exch.sizes) <= set(FIELDS)
        with pytest.raises(ValueError):
            bad = dict(_slot_results(cl))
            bad["vst"] = torch.zeros(1, dtype=torch.uint8)
            exch.exchange(bad, sets[0])
        with pytest.raises(ValueError):
            SlotExchange(WORLD, rank, {"votes": 1}, "cpu", gloo_allgather)
        # bench.py reports throughput against the slowest rank
        assert max_over_ranks(1.5 + rank, "cpu") == 1.5 + (WORLD - 1)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


def _packed_worker(rank, port, errq):
    """bench.py's exchange as it runs on the GPU: ONE packed buffer per slot (pack_layout), the
    slot's fields written in place into its views, SlotExchange({"pack": PB}) all-gathering it, every
    rank unpacking every other rank's blocks with unpack_gathered (bench.py's gathered()); two
    output sets in flight, slot k checked only after slot k + 1 was exchanged into the other set."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        NP = V * N
        layout, PB = pack_layout(NP, V)
        cl = synth.make_cluster(V, N, T, first_validator=owned_validators(rank, V).start)
        shards = [synth.make_cluster(V, N, T, first_validator=owned_validators(r, V).start) for r in range(WORLD)]
        exch = SlotExchange(WORLD, rank, {"pack": PB}, "cpu", gloo_allgather)
        outs = []
        for _ in range(2):
            o = {"pack": torch.full((PB,), 0xAB, dtype=torch.uint8)}
            o.update(pack_views(o["pack"], layout))
            o["xchg"] = exch.gather_buffers()
            outs.append(o)

        def check(slot, o):
            for r in range(WORLD):
                want = _slot_results(shards[r], slot)
                for f in PACK_FIELDS:
                    n = layout[f][1]
                    got = unpack_gathered(o["xchg"]["pack"], layout, PB, WORLD, f)
                    assert got.numel() == WORLD * n
                    assert torch.equal(got[r * n:(r + 1) * n], want[f]), (slot, r, f)

        for slot in range(6):
            o = outs[slot % 2]
            res = _slot_results(cl, slot)
            for f in PACK_FIELDS:  # the slot writes its outputs in place
                o[f].copy_(res[f])
            assert exch.exchange({"pack": o["pack"]}, o["xchg"]) == slot
            if slot:
                check(slot - 1, outs[(slot - 1) % 2])
        check(5, outs[1])
        logs = [None] * WORLD
        dist.all_gather_object(logs, exch.issued)
        assert logs[0] == logs[1] == [(k, "pack") for k in range(6)], logs
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_owned_validators_partition():
    got = [v for r in range(4) for v in owned_validators(r, 5)]
    assert got == list(range(20))


@pytest.mark.parametrize("worker", [_worker, _packed_worker], ids=["fields", "bench_pack"])
def test_sharded_slot_exchange_gloo_world2(worker):
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, port, errq)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
            errs.append("rank timed out")
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_bench_pack_layout():
    """bench.py's one exchanged buffer per slot (shard.pack_layout): the fields tile it exactly, in
    order, with the bitmap rounded up to whole bytes"""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import inspect
    import bench
    # bench.py imports the exchange code inside main (its launcher parent imports no torch code)
    src = inspect.getsource(bench.main)
    assert "from charon_amd.shard import" in src and "pack_layout" in src and "def pack_layout" not in src
    for NP, V in ((1, 1), (12, 3), (1_000_000, 100_000), (875_001, 125_000)):
        layout, total = pack_layout(NP, V)
        pos = 0
        for f in ("vbits", "tout", "tst", "ast"):
            off, size = layout[f]
            assert off == pos, (NP, V, f)
            pos += size
        assert pos == total and layout["vbits"][1] == (NP + 7) // 8 and layout["tout"][1] == 96 * V

