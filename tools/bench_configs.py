"""Throughput of the other BASELINE configs on one MI355X (the headline C2 line is bench.py).

  C3  models/Transformer (build_transformer(16,16,90,5,10,128,3,8,0.05,64)), B=512
  C5  InformerStackLSQ 8-bit weights (QuantizationStudy/LSQ), B=1024 (bf16 activations)
  full  FullPrecision InformerStack attn="full", e_layers=[4,3] (the TimingAnalysis shape), B=512

Seeded synthetic weights (the golden-case builders), seeded synthetic channel features resident in
HBM. Kernel time is the engine's own HIP events on the launch stream; one JSON line per config.

    python tools/bench_configs.py [--steps 100]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from channelestimationtransformer_amd.flops import informer_flops, transformer_flops  # noqa: E402
from channelestimationtransformer_amd.informer import InformerStack, InformerStackLSQ  # noqa: E402
from channelestimationtransformer_amd.spec import informer_stack_spec, transformer_spec  # noqa: E402
from channelestimationtransformer_amd.transformer import build_transformer  # noqa: E402
from channelestimationtransformer_amd.weights import synthetic_state_dict  # noqa: E402

PEAK = 2500.0


def informer(dev, e_layers, attn, lsq_bits=0):
    args = [16, 16, 16, 90, 10, 5, 5, 128, 8, e_layers, 3, 64, 0.05, attn, "fixed", "gelu", False, True, dev]
    m = InformerStackLSQ(*args, lsq_bits) if lsq_bits else InformerStack(*args)
    spec = m._schema()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(spec, 0).items()},
                      strict=False)
    if lsq_bits:
        m.enable_lsq(lsq_bits)
    return m.eval()


def transformer(dev):
    m = build_transformer(16, 16, 90, 5, 10, 128, 3, 8, 0.05, 64)
    spec = transformer_spec(16, 16, 90, 5, 10, 128, 3, 8, 64)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(spec, 0).items()},
                      strict=False)
    return m.eval()


def time_engine(m, dev, B, steps, warmup=10):
    eng = m.engine(dev)
    g = torch.Generator().manual_seed(7)
    xe = (torch.randn(B, 90, 16, generator=g) / 2 ** 0.5).to(dev)
    xd = torch.cat([xe[:, -10:], torch.zeros(B, 5, 16, device=dev)], 1).contiguous()
    out = torch.empty(B, 5, 16, device=dev)
    if hasattr(eng, "seed") and eng.prob_calls():
        eng.seed(1)
    for _ in range(warmup):
        eng.forward(xe, xd, out)
    torch.cuda.synchronize(dev)
    eng.timing(True)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(steps):
        eng.forward(xe, xd, out)
    ev1.record()
    torch.cuda.synchronize(dev)
    ms, k = eng.timing_read()
    eng.timing(False)
    assert torch.isfinite(out).all()
    return ev0.elapsed_time(ev1) / steps, ms / max(k, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--only", default="", help="run only the configs whose name contains this")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    runs = [
        ("C3 Transformer (full attention, no distil), N=3", lambda: transformer(dev), 512, transformer_flops()),
        ("C5 InformerStackLSQ 8-bit weights, prob+distil, e_layers=[4]", lambda: informer(dev, [4], "prob", 8), 1024,
         informer_flops()),
        ("FullPrecision InformerStack attn=full, e_layers=[4,3]", lambda: informer(dev, [4, 3], "full"), 512,
         informer_flops(e_layers=(4, 3), attn="full")),
    ]
    for name, mk, B, flops in runs:
        if args.only not in name:
            continue
        m = mk()
        step_ms, kern_ms = time_engine(m, dev, B, args.steps)
        tf = flops * B / (kern_ms * 1e-3) / 1e12
        print(json.dumps({"config": name, "batch": B, "seq_per_s": round(B / (step_ms * 1e-3), 1),
                          "ms_per_step": round(step_ms, 4), "kernel_ms": round(kern_ms, 4),
                          "flops_per_seq": flops, "tflops": round(tf, 2), "mfma_frac": round(tf / PEAK, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
