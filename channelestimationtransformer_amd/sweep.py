"""SNR sweep (BASELINE config C4) on the device.

Restates the validation pass ``run_validation`` (FullPrecision/QuantizationAwareTraining.py:86-140)
at every SNR of ``SNR.sbatch`` (:9-13: 12, 14, 16, 18, 20 dB), with the whole data path on the GPU:
``DeviceSeqData.batch`` (window, channelnorm, noise, LoadBatch, decoder input) → fused forward →
``NMSE_Split`` accumulated on the device.  The loader semantics are ``DataLoader(shuffle=True,
drop_last=True)``: one seeded permutation per SNR, whole batches only, and the reported loss is the
mean of the per-batch ratios (``loss / len(val_dataloader)``).

Multi-GPU (config C4: a reference batch of 4096 = 8 × 512 sharded over 8 GPUs):
``python -m channelestimationtransformer_amd.sweep --gpus N`` starts N ranks itself (or run it under
torchrun).  Reference batch i is the N shards of ``--batch`` sequences the ranks take from the loader's
permutation at step i.  Each rank keeps the raw fp64 NMSE_Split sums of its shard per step; at the end
of an SNR one all_reduce turns them into each global batch's ratio (``NMSE_Split_cuda`` over all
N × batch predictions) and one all_gather collates the last batch's predictions on rank 0, which
reduces NMSE_Split over them and checks the all-reduced value (no collective in the data path).

Data: ``--dataset`` (a ``.npy`` complex ``[N, slots, 2, 4]``, or a ``.pt`` tensor read with
``weights_only=True``) or, by default, seeded Jakes channels generated on the device.  Weights:
``--checkpoint`` (a reference ``.pt``, see checkpoint.py) or the seeded synthetic recipe.
Prints one JSON line per SNR on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np

# the reference configuration (FullPrecision/config.py:4-35) and the callers' positional call
CONFIG = dict(enc_in=16, dec_in=16, c_out=16, seq_len=90, label_len=10, pred_len=5, factor=5, d_model=128,
              n_heads=8, e_layers=[4], d_layers=3, d_ff=64, dropout=0.05, attn="prob", embed="fixed",
              activation="gelu", output_attention=False, distil=True)


def build_model(device, checkpoint=None, weight_seed=0):
    import torch

    from .checkpoint import load_checkpoint
    from .informer import InformerStack
    from .spec import informer_stack_spec
    from .weights import synthetic_state_dict

    c = CONFIG
    m = InformerStack(c["enc_in"], c["dec_in"], c["c_out"], c["seq_len"], c["label_len"], c["pred_len"], c["factor"],
                      c["d_model"], c["n_heads"], c["e_layers"], c["d_layers"], c["d_ff"], c["dropout"], c["attn"],
                      c["embed"], c["activation"], c["output_attention"], c["distil"], device)
    if checkpoint:
        state = load_checkpoint(checkpoint)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in state.items()}, strict=False)
    else:
        spec = informer_stack_spec(16, 16, 16, 128, 8, [4], 3, 64, freq="gelu")
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(spec, weight_seed).items()})
    return m.eval()


def load_dataset(path):
    import torch

    if path.endswith(".npy"):
        return np.load(path, allow_pickle=False)
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(obj, torch.Tensor):
        raise ValueError(f"{path}: expected a complex tensor [N, slots, Nr, Nt]")
    return obj


def run_snr_point(step, n_batches, T, world=1, rank=0, dist=None, nmse_fn=None, device=None, synchronize=None):
    """One SNR of the sweep, with the engine abstracted away (so the collation runs on CPU under gloo too).

    ``step(i, sums_row)`` runs reference batch i of this rank (its shard of ``world`` shards) and writes
    that shard's raw NMSE_Split sums (float64 [2, T]: Σ(x − x̂)², Σx̂²) into ``sums_row``; it returns the
    shard's (predictions, labels).  After the loop one all_reduce gives every batch's ratio over the
    whole global batch (``NMSE_Split_cuda`` over all N × batch predictions), their mean is
    ``run_validation``'s ``loss / len(loader)`` (QuantizationAwareTraining.py:122,138), and rank 0
    checks NMSE_Split over the all-gathered last predictions (``nmse_fn``) against the all-reduced sums.
    Returns {nmse [T] numpy, ratios [n_batches, T] numpy, seconds (max over ranks), check}."""
    import torch

    from .sharding import check_gathered_nmse, collate_step_sums, gather_predictions

    sync = synchronize or (lambda: None)
    sums = torch.zeros(n_batches, 2, T, dtype=torch.float64, device=device)
    sync()
    t0 = time.perf_counter()
    out = lab = None
    for i in range(n_batches):
        out, lab = step(i, sums[i])
    sync()
    dt = time.perf_counter() - t0
    if dist is not None and world > 1:
        t = torch.tensor([dt], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ratios, nmse = collate_step_sums(sums, world)
    preds, labels = gather_predictions(out, world), gather_predictions(lab, world)
    check = None
    if rank == 0 and nmse_fn is not None:
        g = nmse_fn(torch.cat(preds).contiguous(), torch.cat(labels).contiguous())
        check = check_gathered_nmse(g, ratios[-1])
    return {"nmse": nmse.cpu().numpy(), "ratios": ratios.cpu().numpy(), "seconds": dt, "check": check}


def run_sweep(snrs, batch, batches, dataset=None, n_samples=None, checkpoint=None, seed=0, rank=0, world=1,
              device=None, dist=None, capture=None):
    """Yields one result dict per SNR (identical on every rank).

    ``capture(snr, i, x_enc, x_dec, out, label)``, if given, sees every batch this rank ran (device
    tensors, valid until the next batch): the tests check the sweep's NMSE and predictions against the
    oracle with it.  The ProbSparse draws are the native stream seeded with ``1 + seed``, one forward's
    worth per batch in order."""
    import torch

    from .engine import nmse_split
    from .pipeline import DeviceSeqData, synth_channels

    c = CONFIG
    model = build_model(device, checkpoint)
    eng = model.engine(device)
    eng.seed(1 + seed)                     # ProbSparse draws: the torch.randint stream, natively
    if dataset is None:
        n = n_samples or batch * batches * world
        dataset = synth_channels(n, slots=100, seed=1234 + seed, device=device)
    data = DeviceSeqData(dataset, c["seq_len"], c["pred_len"], label_len=c["label_len"], device=device)
    per_epoch = len(data) // (batch * world)      # drop_last over the global batch
    n_batches = min(batches, per_epoch) if batches else per_epoch
    if n_batches == 0:
        raise ValueError(f"dataset of {len(data)} samples holds no whole batch of {batch} x {world} ranks")
    F = data.features
    bufs = (torch.empty(batch, c["seq_len"], F, device=device),
            torch.empty(batch, c["label_len"] + c["pred_len"], F, device=device),
            torch.empty(batch, c["pred_len"], F, device=device))
    out = torch.empty(batch, c["pred_len"], c["c_out"], device=device)
    stream = torch.cuda.current_stream(device).cuda_stream
    for k, snr in enumerate(snrs):
        g = torch.Generator().manual_seed(seed * 1000 + k)
        perm = torch.randperm(len(data), generator=g).to(torch.int32).to(device)   # the loader's shuffle

        def step(i, sums_row):
            off = (i * world + rank) * batch
            xe, xd, lb = data.batch(idx=perm[off:off + batch], seed=seed, counter=(k << 32) + i * world + rank,
                                    snr=snr, out=bufs, stream=stream)
            eng.forward_nmse(xe, xd, out, lb, None, sums_row, stream)   # forward + NMSE_Split, one launch
            if capture is not None:
                capture(snr, i, xe, xd, out, lb)
            return out, lb

        r = run_snr_point(step, n_batches, c["pred_len"], world, rank, dist, lambda p, y: nmse_split(p, y), device,
                          lambda: torch.cuda.synchronize(device))
        nmse = r["nmse"]
        seqs = n_batches * batch * world
        yield {"snr": snr, "nmse": [float(v) for v in nmse], "nmse_db": [round(float(10 * np.log10(v)), 4) for v in nmse],
               "nmse_db_mean": round(float(10 * np.log10(nmse.mean())), 4), "batches": n_batches,
               "global_batch": batch * world, "sequences": seqs, "seconds": round(r["seconds"], 4),
               "seq_per_s": round(seqs / r["seconds"], 1), "world": world,
               "nmse_gathered_vs_allreduced_rel": r["check"], "kernel_path": eng.last_path()}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--snr", type=float, nargs="+", default=[12, 14, 16, 18, 20])
    ap.add_argument("--gpus", type=int, default=1, help="ranks to start (one process per GPU)")
    ap.add_argument("--batch", type=int, default=512, help="sequences per rank per step (the reference batch is "
                                                            "--batch x ranks)")
    ap.add_argument("--batches", type=int, default=8, help="batches per rank per SNR (0: one epoch)")
    ap.add_argument("--samples", type=int, default=None, help="synthetic dataset size (default: exactly the batches)")
    ap.add_argument("--dataset", default=None)
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args(argv)
    if args.gpus > 1 and "RANK" not in os.environ:
        import sys

        from .sharding import spawn_ranks

        rest = list(argv) if argv is not None else sys.argv[1:]
        raise SystemExit(spawn_ranks(args.gpus, ["channelestimationtransformer_amd.sweep"] + rest, module=True))

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)
    ds = load_dataset(args.dataset) if args.dataset else None
    for res in run_sweep(args.snr, args.batch, args.batches, ds, args.samples, args.checkpoint, args.seed, rank, world,
                         dev, dist):
        if rank == 0:
            print(json.dumps(res), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
