"""Validator sharding across ranks and the slot's one exchange step.

Validators are independent: rank r of N owns validators [r*V, (r+1)*V) of the node's cluster
(weak scaling, every rank V validators), and every partial signature, ThresholdAggregate and
verdict of a validator stays on its rank's GPU.  The only cross-GPU traffic is one all-gather per
slot of (i) the verdict byte of every partial, (ii) the 96-byte aggregate and (iii) the status byte
of every validator, so that every rank holds the node's result in validator order (RCCL over xGMI
on the GPU box; gloo on CPU in tests/test_shard.py).

Plain torch.distributed: the reference's exchange step is charon's sigagg -> bcast fan-out
(core/sigagg/sigagg.go:56-63 hands each aggregate to the broadcaster), which this replaces
within a node.
"""

from __future__ import annotations

import torch
import torch.distributed as dist


def owned_validators(rank: int, validators_per_rank: int) -> range:
    """Global validator indices owned by `rank` (contiguous blocks, rank order)."""
    return range(rank * validators_per_rank, (rank + 1) * validators_per_rank)


class SlotExchange:
    """Gather buffers for one slot's results; `exchange` fills them on every rank.

    vst: uint8[NP] verdicts of the rank's partials (NP = V*n), tout: uint8[V*96] aggregates,
    tst: uint8[V] aggregate statuses.  After `exchange`, `vst_all[r*NP:(r+1)*NP]` is rank r's
    block, i.e. the arrays are in global validator order.
    """

    def __init__(self, world: int, V: int, n: int, device):
        self.world, self.V, self.n = world, V, n
        self.vst_all = torch.empty(world * V * n, dtype=torch.uint8, device=device)
        self.tout_all = torch.empty(world * V * 96, dtype=torch.uint8, device=device)
        self.tst_all = torch.empty(world * V, dtype=torch.uint8, device=device)

    def exchange(self, vst: torch.Tensor, tout: torch.Tensor, tst: torch.Tensor, group=None) -> None:
        if vst.numel() != self.V * self.n or tout.numel() != self.V * 96 or tst.numel() != self.V:
            raise ValueError("slot result shapes do not match the exchange buffers")
        dist.all_gather_into_tensor(self.vst_all, vst, group=group)
        dist.all_gather_into_tensor(self.tout_all, tout, group=group)
        dist.all_gather_into_tensor(self.tst_all, tst, group=group)

    def all_ok(self) -> bool:
        return bool((self.vst_all == 0).all().item() and (self.tst_all == 0).all().item())


def max_over_ranks(seconds: float, device, group=None) -> float:
    """The slowest rank's time (bench.py reports whole-job throughput against it)."""
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
