"""Validator sharding across ranks and the slot's one exchange step.

Validators are independent: rank r of N owns validators [r*V, (r+1)*V) of the node's cluster
(weak scaling, every rank V validators), and every partial signature, ThresholdAggregate and
verdict of a validator stays on its rank's GPU.  The only cross-GPU traffic is one all-gather per
slot of (i) the verdict byte of every partial, (ii) the 96-byte aggregate, (iii) the aggregation
status and (iv) the post-aggregate verification status of every validator, so that every rank
holds the node's result in validator order.

`SlotExchange` is the exchange bench.py runs (RCCL over xGMI through the library's
hbls_allgather_device, `library_allgather`) and tests/test_shard.py runs over gloo on the CPU
(`gloo_allgather`): the all-gather is pluggable, the ordering is not.  With several slots in flight
every exchange goes through ONE exchange stream, in slot order and in a fixed field order, so that
every rank issues its collectives to the communicator in the same sequence (a communicator's
collectives must be issued in the same order on every rank); the producing stream waits for the
exchange before its output set is reused.

The reference's exchange step is charon's sigagg -> bcast fan-out (core/sigagg/sigagg.go:56-63
hands each aggregate to the broadcaster), which this replaces within a node.
"""

from __future__ import annotations

import ctypes
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

FIELDS = ("vst", "vbits", "tout", "tst", "ast", "pack")

# allgather(send, recv, nbytes, stream): gather `nbytes` of `send` from every rank into `recv`
# (rank order), ordered on `stream` (a torch.cuda.Stream, or None on the CPU)
AllGather = Callable[[torch.Tensor, torch.Tensor, int, Optional[object]], None]


def owned_validators(rank: int, validators_per_rank: int) -> range:
    """Global validator indices owned by `rank` (contiguous blocks, rank order)."""
    return range(rank * validators_per_rank, (rank + 1) * validators_per_rank)


def gloo_allgather(send: torch.Tensor, recv: torch.Tensor, nbytes: int, stream=None) -> None:
    """torch.distributed all-gather (gloo on the CPU: the tests' stand-in for RCCL)."""
    del nbytes, stream
    dist.all_gather_into_tensor(recv, send)


def library_allgather(L) -> AllGather:
    """The library's RCCL all-gather over xGMI (hbls_allgather_device) on the exchange stream."""

    def ag(send, recv, nbytes, stream):
        sp = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
        rc = L.hbls_allgather_device(ctypes.c_void_p(send.data_ptr()), ctypes.c_void_p(recv.data_ptr()), nbytes, sp)
        if rc != 0:
            raise RuntimeError("hipbls: " + L.hbls_last_error().decode(errors="replace"))
    return ag


def init_library_comm(L, world: int, rank: int) -> None:
    """The library's RCCL communicator: rank 0 draws the id, the torch.distributed control plane
    (gloo) carries it to the other ranks, every rank joins (hbls_comm_init)."""
    idb = np.zeros(L.hbls_comm_id_bytes(), dtype=np.uint8)
    if rank == 0 and L.hbls_comm_unique_id(ctypes.c_void_p(idb.ctypes.data)) != 0:
        raise RuntimeError("hipbls: " + L.hbls_last_error().decode(errors="replace"))
    if world > 1:
        obj = [idb.tobytes()]
        dist.broadcast_object_list(obj, src=0)
        idb = np.frombuffer(obj[0], dtype=np.uint8).copy()
    if L.hbls_comm_init(world, rank, ctypes.c_void_p(idb.ctypes.data)) != 0:
        raise RuntimeError("hipbls: " + L.hbls_last_error().decode(errors="replace"))


class SlotExchange:
    """All-gather of one slot's results per call, in a fixed issue order.

    sizes: bytes per rank of each field (vst = V*n verdict bytes or vbits = their ceil(V*n/8)-byte
    verify bitmap, tout = V*96 aggregates, tst / ast = V statuses; pack = bench.py's one buffer of
    vbits | tout | tst | ast, one all-gather per slot).  `gather_buffers()` makes one set of receive buffers (one per slot in flight);
    `exchange(outs, recv, producer)` gathers the rank's outputs `outs` into `recv` on the exchange
    stream after `producer` (the slot's stream) has written them, and makes `producer` wait for the
    gather.  `issued` logs (slot sequence number, field) in issue order: identical on every rank.
    """

    def __init__(self, world: int, rank: int, sizes: Dict[str, int], device, allgather: AllGather,
                 stream=None):
        unknown = set(sizes) - set(FIELDS)
        if unknown:
            raise ValueError(f"unknown exchange fields {sorted(unknown)}")
        self.world, self.rank, self.device = world, rank, device
        self.sizes = {f: int(sizes[f]) for f in FIELDS if f in sizes}
        self.allgather = allgather
        self.stream = stream
        self.seq = 0
        self.issued: List[Tuple[int, str]] = []

    def gather_buffers(self) -> Dict[str, torch.Tensor]:
        return {f: torch.empty(self.world * n, dtype=torch.uint8, device=self.device) for f, n in self.sizes.items()}

    def exchange(self, outs: Dict[str, torch.Tensor], recv: Dict[str, torch.Tensor], producer=None) -> int:
        for f, n in self.sizes.items():
            if outs[f].numel() != n or recv[f].numel() != self.world * n:
                raise ValueError(f"slot result '{f}' does not match the exchange buffers")
        if self.stream is not None:
            done = torch.cuda.Event()
            done.record(producer)
            self.stream.wait_event(done)
        for f, n in self.sizes.items():
            self.allgather(outs[f], recv[f], n, self.stream)
            self.issued.append((self.seq, f))
        if self.stream is not None:
            back = torch.cuda.Event()
            back.record(self.stream)
            producer.wait_event(back)  # the producer overwrites these outputs only after the gather
        self.seq += 1
        return self.seq - 1

    def block(self, recv: Dict[str, torch.Tensor], field: str, r: int) -> torch.Tensor:
        """Rank r's block of a gathered field."""
        n = self.sizes[field]
        return recv[field][r * n:(r + 1) * n]


PACK_FIELDS = ("vbits", "tout", "tst", "ast")


def pack_layout(NP: int, V: int):
    """The slot's exchanged outputs in ONE buffer (one all-gather per slot):
    field -> (offset, bytes), and the total -- the verify bitmap of NP partials (hbls_status_bitmap,
    rounded up to whole bytes), V 96-byte aggregates, their statuses, their verification
    statuses."""
    nb = (NP + 7) // 8
    layout = {"vbits": (0, nb), "tout": (nb, 96 * V), "tst": (nb + 96 * V, V), "ast": (nb + 97 * V, V)}
    return layout, nb + 98 * V


def pack_views(pack: torch.Tensor, layout) -> Dict[str, torch.Tensor]:
    """The fields as views of the slot's pack buffer (the slot writes them in place)."""
    return {f: pack[a:a + b] for f, (a, b) in layout.items()}


def unpack_gathered(gathered_pack: torch.Tensor, layout, total: int, world: int, field: str) -> torch.Tensor:
    """Field `field` of every rank, in rank order, from the all-gathered packs (world x total
    bytes): rank r's block is bytes [r n, (r + 1) n) of the result, n = the field's size."""
    a, b = layout[field]
    return torch.cat([gathered_pack[r * total + a:r * total + a + b] for r in range(world)])


def max_over_ranks(seconds: float, device, group=None) -> float:
    """The slowest rank's time (bench.py reports whole-job throughput against it)."""
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
