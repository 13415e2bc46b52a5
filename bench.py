"""Throughput benchmark of the FullPrecision Informer (BASELINE config C2) on MI355X.

A step = one inference forward of a batch of ``--batch`` (default 512) independent channel
sequences (x_enc [90,16], x_dec [15,16] → out [5,16]) through the fused HIP kernel, with a
fresh torch-compatible ProbSparse index draw (native mt19937, as torch.randint would), plus
the NMSE_Split reduction of that batch on the device (run_validation's
``loss += NMSELossSplit(output, label)``, QuantizationAwareTraining.py:115-122).
Inputs are synthetic channels resident in HBM; weights are the seeded synthetic recipe.

Two batches are in flight per GPU by default (``--inflight 2``): step k runs on engine lane k mod 2, each
lane an engine replica (same weights) with its own HIP stream, input batch, resident sampler chain and
fused-NMSE ticket.  Every step is still one full forward of a 512-sequence batch; the second stream lets the
next batch's workgroups take the CUs the current launch's early finishers free (the launch's tail: per-
workgroup time spread ≈ 11 %) instead of waiting for its slowest workgroup.  ``--inflight 1``
is the one-stream, back-to-back form.

Multi-GPU: ``python bench.py --gpus N`` starts N rank processes itself (torch.distributed.run in a
child process, before anything touches the GPU); the driver may also launch it under torchrun.
One process per GPU, each with its own 512-sequence shard of an N×512 global batch (weak scaling,
no collective in the data path).  Every rank keeps the raw fp64 NMSE_Split sums of its shard per
step; after the timed loop one all_reduce gives each step's ratio over the whole global batch, and
one all_gather collates the last step's predictions on rank 0, which reduces NMSE_Split over them
itself and checks it against the all-reduced sums.  Rank 0 prints ONE JSON line.
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
PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table)
KALONE = 256                  # back-to-back launches of the kernel-alone timing after the timed loop
CFG = dict(enc_in=16, dec_in=16, c_out=16, seq_len=90, label_len=10, pred_len=5, factor=5, d_model=128,
           n_heads=8, e_layers=[4], d_layers=3, d_ff=64, dropout=0.05, attn="prob", embed="fixed",
           activation="gelu", output_attention=False, distil=True)
WORKLOAD = ("FullPrecision InformerStack inference (C2): ProbSparse attn, distil, e_layers=[4], d_layers=3, "
            "d_model=128, n_heads=8, d_ff=64, seq_len=90, label_len=10, pred_len=5")


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


def cpu_baseline(batch: int = 512, reps: int = 5):
    """The reference's own PyTorch CPU forward (oracle/informer_torch.py: the aten ops of
    FullPrecision/InformerModel in eval/no_grad, float32) on this host's cores: median of ``reps``
    forwards at B=512 (the GPU workload) and of 20 at B=1."""
    import torch

    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.rng import draw_indices
    from channelestimationtransformer_amd.spec import informer_stack_spec
    from channelestimationtransformer_amd.weights import synthetic_state_dict
    from oracle.informer_np import InformerConfig, sample_shapes
    from oracle.informer_torch import TorchInformer, host_cpu

    host = host_cpu()
    threads = min(v for v in (host["physical_cores"], host["usable_logical"],
                              int(os.environ.get("OMP_NUM_THREADS", "0")) or None) if v)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        cfg = InformerConfig()
        model = TorchInformer(cfg, synthetic_state_dict(informer_stack_spec(16, 16, 16, 128, 8, [4], 3, 64,
                                                                            freq="gelu"), 0), dtype=torch.float32)
        shapes = sample_shapes(cfg)

        def med(b, n, warm):
            xe, xd, _ = make_batch(b, seed=99)
            xe, xd = torch.from_numpy(xe), torch.from_numpy(xd)
            ts = []
            for i in range(warm + n):
                idx = draw_indices(shapes, seed=i)
                t0 = time.perf_counter()
                model.forward(xe, xd, idx)
                if i >= warm:
                    ts.append(time.perf_counter() - t0)
            return float(np.median(ts))

        t_big = med(batch, reps, 1)
        t_one = med(1, 20, 3)
    finally:
        torch.set_num_threads(prev)
    return {"value": round(batch / t_big, 1), "unit": "seq/s", "cores": threads, "kind": "port",
            "sample": f"median of {reps} forwards at B={batch} ({t_big * 1e3:.0f} ms each) of the reference's torch "
                      f"CPU forward (oracle/informer_torch.py, float32, eval/no_grad, {threads} threads)",
            "b1_seq_per_s": round(1.0 / t_one, 1), "cpu_model": host["model"],
            "cores_note": "threads = min(physical cores, usable logical CPUs, OMP_NUM_THREADS): a one-GPU job on "
                          "the 8-GPU box is given 16 CPUs (OMP_NUM_THREADS=16), this GPU's share of the host",
            "host_physical_cores": host["physical_cores"], "host_usable_logical": host["usable_logical"]}


def load_traffic(profile_dir, kernel):
    """HBM bytes per launch of `kernel` from the newest round's committed rocprofv3 PMC summary
    (profiles/rNN/pmc_traffic.json; None if it was collected on another kernel variant), and the file
    it came from."""
    rounds = sorted((d for d in os.listdir(profile_dir) if d.startswith("r") and d[1:].isdigit()),
                    reverse=True) if os.path.isdir(profile_dir) else []
    for r in rounds:
        path = os.path.join(profile_dir, r, "pmc_traffic.json")
        if not os.path.exists(path):
            continue
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            return None, None
        if kernel not in (d.get("kernel") or ""):
            return None, None
        return d.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    return None, None


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--settle-s", type=float, default=1.0,
                    help="keep warming up (untimed) until this many seconds have passed, so the GPU clock has "
                         "settled even with a short --warmup")
    ap.add_argument("--batch", type=int, default=512, help="sequences per GPU per step")
    ap.add_argument("--inflight", type=int, default=2,
                    help="batches in flight per GPU: step k runs on engine lane k mod N, each lane an engine "
                         "replica with its own HIP stream, inputs, sampler chain and NMSE ticket (every step "
                         "is still one full B-sequence forward; 1 = one stream, back-to-back launches)")
    ap.add_argument("--snr", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sampler", choices=("device", "host"), default="device",
                    help="where the native ProbSparse draws run (identical streams; DESIGN §3.3)")
    ap.add_argument("--nmse", choices=("fused", "separate"), default="fused",
                    help="NMSE_Split in the forward's epilogue (cet_forward_nmse) or as its own launch")
    ap.add_argument("--collation-selftest", action="store_true",
                    help="CPU/gloo rehearsal of the multi-rank spawn and NMSE collation (no GPU, no engine)")
    return ap.parse_args(argv)


def collate_and_report(sums, out_last, lab, world, rank, nmse_fn):
    """After the timed loop: all_reduce the per-step sums, all_gather the last predictions on rank 0
    and check NMSE_Split over them against the all-reduced sums of the same step."""
    import torch

    from channelestimationtransformer_amd.sharding import check_gathered_nmse, collate_step_sums, gather_predictions

    ratios, nmse = collate_step_sums(sums, world)
    preds = gather_predictions(out_last, world)
    labels = gather_predictions(lab, world)
    check = None
    if rank == 0:
        g = nmse_fn(torch.cat(preds).contiguous(), torch.cat(labels).contiguous())
        check = check_gathered_nmse(g, ratios[-1])
    return nmse.cpu().numpy(), check


def selftest(args, world, rank):
    """--collation-selftest: the multi-rank launch and the exact collation code of the GPU run, on CPU
    with gloo and seeded stand-in predictions (no kernel runs; nothing is timed)."""
    import torch
    import torch.distributed as dist

    from channelestimationtransformer_amd.sharding import nmse_split_torch

    if world > 1:
        dist.init_process_group("gloo")
    g = torch.Generator().manual_seed(1234 + 7919 * rank)
    T = CFG["pred_len"]
    lab = torch.randn(args.batch, T, 16, generator=g)
    sums = torch.zeros(args.steps, 2, T, dtype=torch.float64)
    out = None
    for s in range(args.steps):
        out = lab + 0.1 * (s + 1) * torch.randn(args.batch, T, 16, generator=g)
        p = out.double()
        d = lab.double() - p
        sums[s, 0], sums[s, 1] = (d * d).sum((0, 2)), (p * p).sum((0, 2))
    nmse, check = collate_and_report(sums, out, lab, world, rank, nmse_split_torch)
    if rank == 0:
        print(json.dumps({"selftest": "collation", "world": world, "backend": "gloo" if world > 1 else None,
                          "steps": args.steps, "global_batch": args.batch * world,
                          "nmse": [float(v) for v in nmse], "gathered_vs_allreduced_rel": check}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main(argv=None):
    args = parse_args(argv)
    if args.gpus > 1 and "RANK" not in os.environ:
        # start the N ranks ourselves: a fresh process per GPU; nothing here has touched the GPU
        from channelestimationtransformer_amd.sharding import spawn_ranks

        rest = list(argv) if argv is not None else sys.argv[1:]
        raise SystemExit(spawn_ranks(args.gpus, [os.path.abspath(__file__)] + rest))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.collation_selftest:
        return selftest(args, world, rank)

    import torch

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)

    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.engine import nmse_split, nmse_split_sums
    from channelestimationtransformer_amd.flops import informer_flops, io_bytes

    B, T, NL = args.batch, CFG["pred_len"], max(1, args.inflight)
    all_sums = torch.zeros(args.steps + 1, 2, T, dtype=torch.float64, device=dev)   # row `steps`: warm-up
    sums = all_sums[:args.steps]
    lanes = []
    for i in range(NL):
        # lane i: an engine replica (same weights) on its own stream, fed its own synthetic batch
        model = build_model(dev)
        eng = model.engine(dev)
        eng.set_sampler(args.sampler == "host")
        eng.seed(1 + i)             # every rank draws the same index samples per lane (shared across the batch)
        xe_np, xd_np, lab_np = make_batch(B, snr=args.snr, seed=1234 + 7919 * rank + 104729 * i)
        xe = torch.from_numpy(xe_np).to(dev)
        xd = torch.from_numpy(xd_np).to(dev)
        lab = torch.from_numpy(lab_np).to(dev)
        out = torch.empty(B, T, 16, device=dev)
        st = torch.cuda.current_stream(dev) if NL == 1 else torch.cuda.Stream(dev)
        fused = eng.bind_forward_nmse(xe, xd, out, lab, all_sums, st.cuda_stream)
        lanes.append(dict(model=model, eng=eng, xe=xe, xd=xd, lab=lab, out=out, stream=st, fused=fused,
                          xe_np=xe_np, xd_np=xd_np))

    def step(k, lane):
        # forward + NMSE_Split of one batch on `lane`: one launch (the kernel fuses the reduction into its
        # epilogue); k < 0: a warm-up step (its sums go to the spare row)
        ln = lanes[lane % NL]
        if args.nmse == "fused":
            ln["fused"](k if k >= 0 else args.steps)
        else:
            with torch.cuda.stream(ln["stream"]):
                ln["eng"].forward(ln["xe"], ln["xd"], ln["out"], None, ln["stream"].cuda_stream)
                nmse_split_sums(ln["out"], ln["lab"], all_sums[k if k >= 0 else args.steps],
                                stream=ln["stream"].cuda_stream)
    eng = lanes[0]["eng"]

    t_w = time.perf_counter()
    n_warm = 0
    while n_warm < args.warmup or time.perf_counter() - t_w < args.settle_s:
        for _ in range(64 if n_warm >= args.warmup else 1):
            step(-1, n_warm)
            n_warm += 1
        if n_warm >= args.warmup:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k, k)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt_rank = time.perf_counter() - t0
    last = lanes[(args.steps - 1) % NL]   # the lane that ran the last timed step
    out_last = last["out"].clone()        # its predictions, kept for the collation below
    path = eng.last_path()                # the fused kernel the timed steps launched
    if path != "v4":
        raise SystemExit(f"the timed steps ran the {path} path, not the fused v4 kernel")
    kernel_name = eng.last_kernel()       # its instance (the C2 one when the plan is C2's: plan_is_c2)
    # the kernel alone, after the timed loop (roofline.kernel_ms): lane 0's forward launches back to back on
    # its stream with nothing else in flight, one event pair around KALONE launches (the forward only: with
    # --nmse separate the reduction's launch is left out)
    ln0 = lanes[0]
    st0 = ln0["stream"]

    def forward_only():
        if args.nmse == "fused":
            ln0["fused"](args.steps)
        else:
            with torch.cuda.stream(st0):
                ln0["eng"].forward(ln0["xe"], ln0["xd"], ln0["out"], None, st0.cuda_stream)
    for _ in range(16):   # the clock is still at its loaded level: the timed loop just ended
        forward_only()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    ev0.record(st0)
    for _ in range(KALONE):
        forward_only()
    ev1.record(st0)
    torch.cuda.synchronize(dev)
    kern_ms, launches = ev0.elapsed_time(ev1), KALONE
    if eng.last_kernel() != kernel_name:
        raise SystemExit(f"the kernel-alone loop ran {eng.last_kernel()}, the timed steps {kernel_name}")

    per_rank = [dt_rank]
    if dist:
        allt = [torch.zeros(1, dtype=torch.float64, device=dev) for _ in range(world)]
        dist.all_gather(allt, torch.tensor([dt_rank], dtype=torch.float64, device=dev))
        per_rank = [float(t.item()) for t in allt]
    dt = max(per_rank)
    nmse, check = collate_and_report(sums, out_last, last["lab"], world, rank, lambda p, y: nmse_split(p, y))

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
            ln0 = lanes[0]
            eng.set_indices(idx)
            o8 = torch.empty(8, 5, 16, device=dev)
            eng.forward(ln0["xe"][:8].contiguous(), ln0["xd"][:8].contiguous(), o8)
            torch.cuda.synchronize(dev)
            ref, _ = InformerOracle(InformerConfig(), synthetic_state_dict(
                informer_stack_spec(16, 16, 16, 128, 8, [4], 3, 64, freq="gelu"), 0)).forward(
                    ln0["xe_np"][:8], ln0["xd_np"][:8], idx)
            a, r = o8.cpu().numpy().astype(np.float64), ref
            parity = float(np.sum((a - r) ** 2) / np.sum(r ** 2))
        except Exception as exc:  # pragma: no cover - reported, not fatal
            parity = f"error: {exc}"
        traffic, traffic_src = load_traffic(os.path.join(ROOT, "profiles"), kernel_name)
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
            "config": {"workload": WORKLOAD, "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": f"dp{world}", "nmse": args.nmse,
                       "inflight_batches_per_gpu": NL},
            "world": world,
            "backend": "nccl" if world > 1 else None,
            "per_rank_ms_per_step": [round(t / args.steps * 1e3, 4) for t in per_rank],
            "warmup_steps_run": n_warm,
            "nmse_db": [round(float(10 * np.log10(v)), 3) for v in nmse],
            "nmse_gathered_vs_allreduced_rel": check,
            "parity_rel_nmse_vs_oracle": parity,
            "roofline": {"bound": "mfma", "achieved": round(achieved, 3), "peak": PEAK_BF16_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 5),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": kernel_name, "kernel_ms": round(avg_kernel_s * 1e3, 4),
                         "kernel_ms_note": ("the kernel alone: %d back-to-back launches of lane 0 on its stream "
                                            "after the timed loop, nothing else in flight, one HIP event pair "
                                            "around them (independent of --steps; compare the rocprofv3 "
                                            "kernel-trace average in profiles/)" % KALONE),
                         "achieved_from_throughput": round(flops * seqs / dt / 1e12, 3),
                         "frac_effective": round(flops * seqs / dt / 1e12 / PEAK_BF16_TFLOPS, 5),
                         "flops_per_seq": flops, "io_bytes_per_seq": io_bytes(),
                         "hbm_achieved_gbps": round(io_bytes() * B / avg_kernel_s / 1e9, 2)},
        }
        if not args.no_cpu_baseline and world == 1:   # the CPU leg: rank 0 at N=1 only
            res["cpu_baseline"] = cpu_baseline(B)
        print(json.dumps(res), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
