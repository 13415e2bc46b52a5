"""Throughput benchmark of the FullPrecision Informer (BASELINE config C2) on MI355X.

A step = one inference forward of a batch of ``--batch`` (default 512) independent channel
sequences (x_enc [90,16], x_dec [15,16] → out [5,16]) through the fused HIP kernel, with a
fresh torch-compatible ProbSparse index draw (native mt19937, as torch.randint would), plus
the NMSE_Split reduction of that batch accumulated on device (run_validation's
``loss += NMSELossSplit(output, label)``, QuantizationAwareTraining.py:115-122).
Inputs are synthetic channels resident in HBM; weights are the seeded synthetic recipe.

Multi-GPU (launched by torch.distributed.run): one process per GPU, each with its own
512-sequence shard (weak scaling, no collective in the data path); after the timed loop the
per-rank NMSE accumulators are all-reduced and the last step's predictions all-gathered over
RCCL for the NMSE reduction.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "channel-sequences/sec + NMSE(dB), FullPrecision Informer @1/2/4/8 MI355X"
KERNEL_NAMES = {1: "cet::informer_forward<64>", 2: "cet::v2::informer_forward_v2<64>",
                3: "cet::v3::informer_forward_v3<64, false, true>"}
PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table)
CFG = dict(enc_in=16, dec_in=16, c_out=16, seq_len=90, label_len=10, pred_len=5, factor=5, d_model=128,
           n_heads=8, e_layers=[4], d_layers=3, d_ff=64, dropout=0.05, attn="prob", embed="fixed",
           activation="gelu", output_attention=False, distil=True)


def build_model(device):
    import torch

    from channelestimationtransformer_amd.informer import InformerStack
    from channelestimationtransformer_amd.spec import informer_stack_spec
    from channelestimationtransformer_amd.weights import synthetic_state_dict

    c = CFG
    # the callers' 19-positional-argument construction (QuantizationAwareTraining.py:63-83)
    m = InformerStack(c["enc_in"], c["dec_in"], c["c_out"], c["seq_len"], c["label_len"], c["pred_len"], c["factor"],
                      c["d_model"], c["n_heads"], c["e_layers"], c["d_layers"], c["d_ff"], c["dropout"], c["attn"],
                      c["embed"], c["activation"], c["output_attention"], c["distil"], device)
    spec = informer_stack_spec(16, 16, 16, 128, 8, [4], 3, 64, freq="gelu")
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(spec, 0).items()})
    return m.eval()


def cpu_baseline(seconds: float = 12.0, batch: int = 32):
    """The numpy oracle (a restatement of the reference CPU forward, float32) on host cores."""
    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.rng import draw_indices
    from channelestimationtransformer_amd.spec import informer_stack_spec
    from channelestimationtransformer_amd.weights import synthetic_state_dict
    from oracle.informer_np import InformerConfig, InformerOracle, sample_shapes

    cfg = InformerConfig()
    orc = InformerOracle(cfg, synthetic_state_dict(informer_stack_spec(16, 16, 16, 128, 8, [4], 3, 64, freq="gelu"), 0),
                         dtype=np.float32)
    xe, xd, _ = make_batch(batch, seed=99)
    shapes = sample_shapes(cfg)
    orc.forward(xe, xd, draw_indices(shapes, seed=0))   # warm-up
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        orc.forward(xe, xd, draw_indices(shapes, seed=n))
        n += 1
    dt = time.perf_counter() - t0
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": round(n * batch / dt, 2), "unit": "seq/s", "cores": threads, "kind": "port",
            "sample": f"{n} forwards of B={batch} (numpy oracle, float32, {dt:.1f}s)"}


def load_traffic(profile_dir, kernel):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 PMC summary (None if the summary
    was collected on another kernel variant)."""
    path = os.path.join(profile_dir, "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        if kernel not in (d.get("kernel") or ""):
            return None
        return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--batch", type=int, default=512, help="sequences per GPU per step")
    ap.add_argument("--snr", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--variant", type=int, default=3,
                    help="fused-kernel generation (1: LDS-resident, 2: 4-wave register-resident, 3: 8-wave)")
    ap.add_argument("--sampler", choices=("device", "host"), default="device",
                    help="where the native ProbSparse draws run (identical streams; DESIGN §3.3)")
    ap.add_argument("--nmse-stream", choices=("same", "side"), default="same",
                    help="side: NMSE_Split of step n runs on a second stream, overlapping forward n+1 "
                         "(predictions double-buffered)")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit("for --gpus N>1 launch with: python -m torch.distributed.run --nproc-per-node N "
                         "--master-addr 127.0.0.1 bench.py --gpus N")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)

    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.engine import nmse_split
    from channelestimationtransformer_amd.flops import informer_flops, io_bytes

    model = build_model(dev)
    eng = model.engine(dev)
    eng.set_variant(args.variant)
    eng.set_sampler(args.sampler == "host")
    eng.seed(1)                 # every rank draws the same index samples (shared across the batch)
    B = args.batch
    xe_np, xd_np, lab_np = make_batch(B, snr=args.snr, seed=1234 + 7919 * rank)
    xe = torch.from_numpy(xe_np).to(dev)
    xd = torch.from_numpy(xd_np).to(dev)
    lab = torch.from_numpy(lab_np).to(dev)
    outs = [torch.empty(B, 5, 16, device=dev) for _ in range(2)]
    acc = torch.zeros(5, device=dev)
    main_s = torch.cuda.current_stream(dev)
    stream = main_s.cuda_stream
    side_s = torch.cuda.Stream(dev) if args.nmse_stream == "side" else None
    fwd_done = torch.cuda.Event()
    nmse_done = [torch.cuda.Event(), torch.cuda.Event()]
    n_step = [0]

    def step():
        if side_s is None:
            eng.forward(xe, xd, outs[0], None, stream)
            nmse_split(outs[0], lab, acc, accumulate=True, stream=stream)
            return
        i = n_step[0] & 1
        n_step[0] += 1
        main_s.wait_event(nmse_done[i])       # NMSE of step n-2 has finished reading outs[i]
        eng.forward(xe, xd, outs[i], None, stream)
        fwd_done.record(main_s)
        side_s.wait_event(fwd_done)
        nmse_split(outs[i], lab, acc, accumulate=True, stream=side_s.cuda_stream)
        nmse_done[i].record(side_s)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    acc.zero_()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    eng.timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    kern_ms, launches = eng.timing_read()
    eng.timing(False)
    from channelestimationtransformer_amd.sharding import collate_nmse, gather_predictions

    dt_t = torch.tensor([dt], device=dev, dtype=torch.float64)
    if dist:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    nmse = collate_nmse(acc, args.steps, world).cpu().numpy()     # RCCL all_reduce of NMSE partials
    out = outs[(n_step[0] - 1) & 1] if side_s is not None else outs[0]
    gather_predictions(out, world)                                # RCCL all_gather of the last predictions

    if rank == 0:
        flops = informer_flops()
        seqs = B * world * args.steps
        avg_kernel_s = kern_ms / 1e3 / max(launches, 1)
        achieved = flops * B / avg_kernel_s / 1e12
        # parity spot check of this very engine against the CPU oracle (8 sequences, fixed draws)
        parity = None
        try:
            from channelestimationtransformer_amd.rng import draw_indices
            from channelestimationtransformer_amd.spec import informer_stack_spec
            from channelestimationtransformer_amd.weights import synthetic_state_dict
            from oracle.informer_np import InformerConfig, InformerOracle, sample_shapes

            idx = draw_indices(sample_shapes(InformerConfig()), seed=5)
            eng.set_indices(idx)
            o8 = torch.empty(8, 5, 16, device=dev)
            eng.forward(xe[:8].contiguous(), xd[:8].contiguous(), o8)
            torch.cuda.synchronize(dev)
            ref, _ = InformerOracle(InformerConfig(), synthetic_state_dict(
                informer_stack_spec(16, 16, 16, 128, 8, [4], 3, 64, freq="gelu"), 0)).forward(xe_np[:8], xd_np[:8], idx)
            a, r = o8.cpu().numpy().astype(np.float64), ref
            parity = float(np.sum((a - r) ** 2) / np.sum(r ** 2))
        except Exception as exc:  # pragma: no cover - reported, not fatal
            parity = f"error: {exc}"
        res = {
            "metric": METRIC,
            "value": round(seqs / dt, 1),
            "unit": "seq/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (seeded Jakes channels, SNR %g dB; seeded synthetic weights)" % args.snr,
            "config": {"workload": "FullPrecision InformerStack inference (C2): ProbSparse attn, distil, "
                                   "e_layers=[4], d_layers=3, d_model=128, n_heads=8, d_ff=64, seq_len=90, "
                                   "label_len=10, pred_len=5",
                       "batch_per_gpu": B, "global_batch": B * world, "parallelism": f"dp{world}",
                       "nmse_stream": args.nmse_stream},
            "nmse_db": [round(float(10 * np.log10(v)), 3) for v in nmse],
            "parity_rel_nmse_vs_oracle": parity,
            "roofline": {"bound": "mfma", "achieved": round(achieved, 3), "peak": PEAK_BF16_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 5),
                         "traffic": load_traffic(os.path.join(ROOT, "profiles"), KERNEL_NAMES[args.variant]),
                         "kernel": KERNEL_NAMES[args.variant], "kernel_ms": round(avg_kernel_s * 1e3, 4),
                         "flops_per_seq": flops, "io_bytes_per_seq": io_bytes(),
                         "hbm_achieved_gbps": round(io_bytes() * B / avg_kernel_s / 1e9, 2)},
        }
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        print(json.dumps(res), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
