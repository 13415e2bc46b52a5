"""Batch sharding across GPUs and the NMSE collation step.

Every channel sequence is independent, so a global batch is split into contiguous per-rank
shards with no data-path collective.  The only exchanges happen after the timed loop:

* ``collate_step_sums``: every rank kept, per step, the raw fp64 NMSE_Split sums of its shard
  (Σ(x−x̂)², Σx̂² per prediction step, ``cet_nmse_split_sums``).  One ``all_reduce`` adds them, so
  each step's ratio is the reference's ``NMSE_Split_cuda`` over the WHOLE global batch of that step
  (``FullPrecision/metrics.py:26-30``), and the steps are averaged as ``run_validation`` averages
  per-batch ratios (``QuantizationAwareTraining.py:122,138``);
* ``gather_predictions``: the north star's RCCL all-gather — rank 0 collates the last step's
  predictions (and labels) of every rank and reduces NMSE_Split over them itself, which must agree
  with the all-reduced sums of that step (``check_gathered_nmse``).

bench.py and the SNR sweep (``sweep.run_snr_point``) both collate this way.  A reference batch of the
multi-GPU sweep is the N ranks' shards of one step (C4: 8 × 512 = 4096 sequences per batch), so its
NMSE is NMSE_Split over the whole global batch, as the reference computes it over one 4096 batch.

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


def collate_step_sums(sums, world: int, group=None):
    """``sums`` float64 [steps, 2, T] of this rank's shards → (per-step global ratios [steps, T], their mean [T]).

    After the all_reduce every rank holds the global Σ(x−x̂)² and Σx̂² of every step."""
    import torch.distributed as dist

    if world > 1:
        dist.all_reduce(sums, group=group)
    ratios = sums[:, 0, :] / sums[:, 1, :]
    return ratios, ratios.mean(0)


def gather_predictions(pred, world: int, group=None) -> List:
    """All-gather equally sized per-rank prediction shards (rank order)."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return [pred]
    out = [torch.empty_like(pred) for _ in range(world)]
    dist.all_gather(out, pred.contiguous(), group=group)
    return out


def nmse_split_torch(pred, label):
    """``NMSE_Split_cuda(x_hat=pred, x=label)`` in float64 torch ops (FullPrecision/metrics.py:26-30):
    Σ_{b,f}(x − x̂)² / Σ_{b,f} x̂² per prediction step.  Used where no HIP device is present."""
    p = pred.double()
    d = label.double() - p
    return (d * d).sum((0, 2)) / (p * p).sum((0, 2))


def check_gathered_nmse(gathered_nmse, last_step_ratio, rtol: float = 1e-5) -> float:
    """Largest relative difference between NMSE_Split of the gathered predictions (rank 0) and the
    all-reduced sums of the same step; raises if it exceeds ``rtol``."""
    import torch

    g = torch.as_tensor(gathered_nmse, dtype=torch.float64).cpu()
    r = torch.as_tensor(last_step_ratio, dtype=torch.float64).cpu()
    diff = float(((g - r).abs() / r.abs()).max())
    if not diff <= rtol:
        raise AssertionError(f"gathered-prediction NMSE {g.tolist()} != all-reduced {r.tolist()} (rel {diff:.2e})")
    return diff


def free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, target: List[str], module: bool = False) -> int:
    """Run ``target`` (a script path + its args, or a module name + args) as ``n`` ranks of ONE node
    through ``torch.distributed.run`` in a child process, and return its exit code.

    The caller must not have touched the GPU: every rank is a fresh process (one per GPU) started by
    the launcher, never an exec of a process that initialised HIP."""
    import os
    import subprocess
    import sys

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}"]
    cmd += (["--module"] if module else []) + list(target)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this host driver
    return subprocess.call(cmd, env=env)
