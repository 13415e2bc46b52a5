"""Batch sharding across GPUs and the NMSE collation step.

Every channel sequence is independent, so a global batch is split into contiguous per-rank
shards with no data-path collective.  The only exchanges are at the end:

* ``collate_nmse``: per-rank NMSE_Split accumulators (sum over that rank's reference batches)
  all-reduced, then divided by the number of batches — the reference's mean of per-batch
  ratios (``run_validation``, QuantizationAwareTraining.py:122,138) when every rank holds
  whole reference batches;
* ``gather_predictions``: all-gather of the per-rank predictions ``[b, pred_len, c_out]`` so
  rank 0 can reduce NMSE over the whole global batch (the north star's "RCCL all-gather of
  predictions").

Works with any torch.distributed backend: ``nccl`` (RCCL over xGMI) on the GPU node, ``gloo``
in the CPU tests.
"""
from __future__ import annotations

from typing import List, Tuple


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, stop) of ``rank``'s shard; sizes differ by at most one."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def collate_nmse(acc, n_batches_per_rank: int, world: int, group=None):
    """Global mean of per-batch NMSE ratios from per-rank sums (all_reduce, SUM)."""
    import torch.distributed as dist

    if world > 1:
        dist.all_reduce(acc, group=group)
    return acc / float(n_batches_per_rank * world)


def gather_predictions(pred, world: int, group=None) -> List:
    """All-gather equally sized per-rank prediction shards (rank order)."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return [pred]
    out = [torch.empty_like(pred) for _ in range(world)]
    dist.all_gather(out, pred.contiguous(), group=group)
    return out
