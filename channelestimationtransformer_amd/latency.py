"""Batch-1 latency mode: the TimingAnalysis harness on the fused engine.

Restates ``run_validation`` of TimingAnalysis/TrainInformer.py:91-151 for the config of
TimingAnalysis/config.py:4-35 (batch 1, attn="full", e_layers=[4, 3], d_layers=3, SNR 80):
each repetition builds one sample's encoder/decoder input on the device, then times ONLY the
model call between two events on the compute stream (``starter.record(); model(...);
ender.record()``), 20 warm-up calls, 1000 timed.  The model call is the drop-in
``InformerStack.forward`` — Python dispatch included, as in the reference's measurement.

The reference's published series (TrainInformer.py:226-234) sweep
``e_layers = [k]``, k = 1..5 at d_layers 3, then d_layers 1..5 at e_layers [5]; ``--series``
runs them.  The harness's own "Mean time" divides the sum of 999 filled slots by 1000
(``timings[batch_idx - 20]`` with ``batch_idx > 20``); ``harness_mean_ms`` reproduces that
quirk next to the true mean.

``--sweep`` runs the whole cumulative sweep of TrainInformer.py:226-264 (each loop leaves its last
value in the config for the next): e_layers [1..5], d_layers 1..5, n_heads 1..5 (d_keys =
d_model // n_heads), d_ff 64..1024, d_model 64..1024, seq_len 12..72, pred_len 1..9, label_len
5..25.  Shapes outside d_model 128 / 8 heads / d_ff ≤ 128 run on the layer-wise engine (fp32).

    python -m channelestimationtransformer_amd.latency [--series | --sweep] [--reps 1000]
"""
from __future__ import annotations

import argparse
import json

import numpy as np

CONFIG = dict(enc_in=16, dec_in=16, c_out=16, seq_len=90, label_len=10, pred_len=5, factor=5, d_model=128, n_heads=8,
              e_layers=[4, 3], d_layers=3, d_ff=64, dropout=0.05, attn="full", embed="fixed", activation="gelu",
              output_attention=False, distil=True, SNR=80)


def build(cfg, device, weight_seed=0):
    import torch

    from .informer import InformerStack
    from .spec import informer_stack_spec
    from .weights import synthetic_state_dict

    c = cfg
    m = InformerStack(c["enc_in"], c["dec_in"], c["c_out"], c["seq_len"], c["label_len"], c["pred_len"], c["factor"],
                      c["d_model"], c["n_heads"], c["e_layers"], c["d_layers"], c["d_ff"], c["dropout"], c["attn"],
                      c["embed"], c["activation"], c["output_attention"], c["distil"], device)
    spec = informer_stack_spec(c["enc_in"], c["dec_in"], c["c_out"], c["d_model"], c["n_heads"], c["e_layers"],
                               c["d_layers"], c["d_ff"], freq=c["activation"])
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(spec, weight_seed).items()})
    return m.eval()


def measure(cfg, device, reps=1000, warmup=20, seed=0):
    """Latency statistics (ms) of one config, harness protocol."""
    import torch

    from .pipeline import DeviceSeqData, synth_channels

    c = cfg
    model = build(c, device)
    n = reps + warmup + 1
    data = DeviceSeqData(synth_channels(min(n, 4096), slots=100, seed=1234 + seed, device=device), c["seq_len"],
                         c["pred_len"], SNR=c["SNR"], label_len=c["label_len"], device=device)
    starter, ender = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = []
    with torch.no_grad():
        for i in range(n):
            xe, xd, _ = data.batch(B=1, sample_base=i % len(data), seed=seed, counter=i)
            starter.record()
            out = model(xe, range(c["seq_len"]), xd, range(c["pred_len"] + c["label_len"]))
            ender.record()
            if i > warmup:
                torch.cuda.synchronize(device)
                times.append(starter.elapsed_time(ender))
    t = np.asarray(times[:reps - 1])
    if isinstance(out, tuple):     # the callers' positional quirk makes output_attention effective
        out = out[0]
    assert tuple(out.shape) == (1, c["pred_len"], c["c_out"])
    eng = "layerwise" if "fp32" in model.engine(device).precision() else "fused"
    return {"engine": eng, "mean_ms": round(float(t.mean()), 5), "std_ms": round(float(t.std()), 5),
            "p50_ms": round(float(np.median(t)), 5), "p99_ms": round(float(np.percentile(t, 99)), 5),
            "harness_mean_ms": round(float(t.sum() / reps), 5), "reps": int(t.size)}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--reps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--series", action="store_true", help="the published e_layers / d_layers series")
    ap.add_argument("--sweep", action="store_true", help="the whole cumulative TimingAnalysis sweep")
    args = ap.parse_args(argv)

    import torch

    dev = torch.device("cuda", 0)
    runs = [("timing_config", dict(CONFIG))]
    if args.series:
        for e in range(1, 6):
            runs.append((f"e_layers_{e}", dict(CONFIG, e_layers=[e], d_layers=3)))
        for d in range(1, 6):
            runs.append((f"d_layers_{d}", dict(CONFIG, e_layers=[5], d_layers=d)))
    if args.sweep:
        runs = [("timing_config", dict(CONFIG))] + cumulative_sweep(CONFIG)
    for name, cfg in runs:
        res = measure(cfg, dev, args.reps, args.warmup)
        print(json.dumps({"run": name, "batch": 1, "attn": cfg["attn"], "e_layers": cfg["e_layers"],
                          "d_layers": cfg["d_layers"], "n_heads": cfg["n_heads"], "d_ff": cfg["d_ff"],
                          "d_model": cfg["d_model"], "seq_len": cfg["seq_len"], "pred_len": cfg["pred_len"],
                          "label_len": cfg["label_len"], **res}), flush=True)


def cumulative_sweep(base):
    """TimingAnalysis/TrainInformer.py:226-264: every loop modifies the running config in place."""
    cfg = dict(base)
    runs = []
    for key, vals, wrap in (("e_layers", [1, 2, 3, 4, 5], lambda v: [v]), ("d_layers", [1, 2, 3, 4, 5], None),
                            ("n_heads", [1, 2, 3, 4, 5], None), ("d_ff", [64, 128, 256, 512, 1024], None),
                            ("d_model", [64, 128, 256, 512, 1024], None), ("seq_len", [12, 24, 48, 60, 72], None),
                            ("pred_len", [1, 3, 5, 7, 9], None), ("label_len", [5, 10, 15, 20, 25], None)):
        for v in vals:
            cfg[key] = wrap(v) if wrap else v
            runs.append((f"{key}_{v}", dict(cfg)))
    return runs


if __name__ == "__main__":
    main()
