"""world_size-2 gloo test of the multi-GPU sharding/collation logic (runs on CPU).

Each rank predicts its contiguous shard (the CPU oracle stands in for the GPU engine here),
accumulates NMSE_Split, then the collectives of :mod:`channelestimationtransformer_amd.sharding`
— driven through the SNR sweep's own per-SNR loop, ``sweep.run_snr_point`` — must reproduce the
unsharded computation.
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from channelestimationtransformer_amd.sharding import shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


PER_RANK, N_BATCHES = 3, 2   # a global reference batch = world × PER_RANK sequences (C4: 8 × 512)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from channelestimationtransformer_amd.dataset import make_batch
        from channelestimationtransformer_amd.sharding import nmse_split_torch
        from channelestimationtransformer_amd.sweep import run_snr_point
        from golden_util import load_case, oracle_for

        case = load_case("informer_prob_b4")
        orc = oracle_for(case)
        xe, xd, lab = make_batch(world * PER_RANK * N_BATCHES, seed=3)

        def step(i, sums_row):   # this rank's shard of global batch i (sweep.run_sweep's indexing)
            off = (i * world + rank) * PER_RANK
            out, _ = orc.forward(xe[off:off + PER_RANK], xd[off:off + PER_RANK], case.idx)
            p, y = torch.from_numpy(out), torch.from_numpy(lab[off:off + PER_RANK])
            d = y.double() - p.double()
            sums_row[0], sums_row[1] = (d * d).sum((0, 2)), (p.double() ** 2).sum((0, 2))
            return p.float(), y

        r = run_snr_point(step, N_BATCHES, 5, world, rank, dist, nmse_split_torch)
        if rank == 0:
            q.put((r["nmse"], r["ratios"], r["check"]))
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions():
    for total in (0, 1, 7, 512, 4096):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_two_rank_sweep_collation_matches_unsharded():
    """The SNR sweep's per-SNR loop and collation (sweep.run_snr_point: per-rank raw sums, all_reduce,
    all_gather of the last predictions, rank 0's check) at world 2 over gloo: every global batch's
    ratio equals NMSE_Split over that batch's unsharded predictions, and the reported NMSE is their
    mean (run_validation's mean of per-batch ratios)."""
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from channelestimationtransformer_amd.dataset import make_batch
    from golden_util import load_case, oracle_for
    from oracle.metrics_np import nmse_split

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    nmse, ratios, check = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0

    case = load_case("informer_prob_b4")
    orc = oracle_for(case)
    G = 2 * PER_RANK
    xe, xd, lab = make_batch(G * N_BATCHES, seed=3)
    ref_preds, _ = orc.forward(xe, xd, case.idx)
    ref = np.stack([nmse_split(ref_preds[i * G:(i + 1) * G].astype(np.float32), lab[i * G:(i + 1) * G])
                    for i in range(N_BATCHES)])
    np.testing.assert_allclose(ratios, ref, rtol=1e-6)
    np.testing.assert_allclose(nmse, ref.mean(0), rtol=1e-6)
    assert check is not None and check < 1e-5


def test_bench_spawns_its_ranks_and_collates_by_gather():
    """`python bench.py --gpus 2` starts its two ranks itself (torch.distributed.run child, gloo here via
    --collation-selftest): the per-step sums are all-reduced, rank 0 all-gathers the last step's
    predictions and its NMSE_Split over them equals the all-reduced value; the mean of per-step
    global ratios equals the unsharded computation."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--collation-selftest",
                        "--steps", "3", "--batch", "8"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, r.stdout
    res = json.loads(line[0])
    assert res["world"] == 2 and res["backend"] == "gloo" and res["global_batch"] == 16
    assert res["gathered_vs_allreduced_rel"] < 1e-12
    # unsharded reference: the same stand-in predictions of both ranks, one ratio per global step
    T, steps = 5, 3
    labs, outs = [], [[] for _ in range(steps)]
    for rank in range(2):
        g = torch.Generator().manual_seed(1234 + 7919 * rank)
        lab = torch.randn(8, T, 16, generator=g)
        labs.append(lab)
        for s in range(steps):
            outs[s].append(lab + 0.1 * (s + 1) * torch.randn(8, T, 16, generator=g))
    from channelestimationtransformer_amd.sharding import nmse_split_torch

    lab = torch.cat(labs)
    ref = torch.stack([nmse_split_torch(torch.cat(outs[s]), lab) for s in range(steps)]).mean(0)
    np.testing.assert_allclose(res["nmse"], ref.numpy(), rtol=1e-12)


def test_step_sum_collation_two_ranks():
    """collate_step_sums over gloo: global per-step ratios from per-rank sums."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sums_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ratios, nmse = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from channelestimationtransformer_amd.sharding import nmse_split_torch

    preds, labs = _sums_data()
    ref = torch.stack([nmse_split_torch(torch.cat([preds[0][s], preds[1][s]]), torch.cat(labs)) for s in range(4)])
    np.testing.assert_allclose(ratios, ref.numpy(), rtol=1e-12)
    np.testing.assert_allclose(nmse, ref.mean(0).numpy(), rtol=1e-12)


def _sums_data():
    g = torch.Generator().manual_seed(5)
    labs = [torch.randn(6, 5, 16, generator=g) for _ in range(2)]
    preds = [[labs[r] + torch.randn(6, 5, 16, generator=g) for _ in range(4)] for r in range(2)]
    return preds, labs


def _sums_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from channelestimationtransformer_amd.sharding import collate_step_sums

        preds, labs = _sums_data()
        sums = torch.zeros(4, 2, 5, dtype=torch.float64)
        for s in range(4):
            p = preds[rank][s].double()
            d = labs[rank].double() - p
            sums[s, 0], sums[s, 1] = (d * d).sum((0, 2)), (p * p).sum((0, 2))
        ratios, nmse = collate_step_sums(sums, world)
        if rank == 0:
            q.put((ratios.numpy(), nmse.numpy()))
    finally:
        dist.destroy_process_group()
