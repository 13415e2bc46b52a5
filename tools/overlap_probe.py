"""Experiment: do two in-flight C2 batches on two HIP streams (two engines, each with its own
resident sampler chain and fused NMSE ticket) finish K steps sooner than one stream?

python tools/overlap_probe.py [steps]   (GPU; prints one JSON line per arrangement)
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import build_model  # noqa: E402
from channelestimationtransformer_amd.dataset import make_batch  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    dev = torch.device("cuda", 0)
    B, T = 512, 5
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    lanes = []
    for i in range(2):
        m = build_model(dev)
        eng = m.engine(dev)
        eng.seed(1 + i)
        xe_np, xd_np, lab_np = make_batch(B, snr=20.0, seed=1234 + i)
        xe, xd, lab = (torch.from_numpy(a).to(dev) for a in (xe_np, xd_np, lab_np))
        out = torch.empty(B, T, 16, device=dev)
        sums = torch.zeros(steps + 1, 2, T, dtype=torch.float64, device=dev)
        f = eng.bind_forward_nmse(xe, xd, out, lab, sums, streams[i].cuda_stream)
        lanes.append((m, eng, f))

    def run(n_streams, k):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for s in range(k):
            lanes[s % n_streams][2](s // n_streams if s < steps else steps)
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    for _ in range(3):
        run(1, 200)
        run(2, 200)
    for rep in range(3):
        for n in (1, 2):
            dt = run(n, steps)
            print(json.dumps({"streams": n, "steps": steps, "ms_per_step": round(dt / steps * 1e3, 4),
                              "seq_per_s": round(steps * B / dt, 1), "rep": rep}), flush=True)


if __name__ == "__main__":
    main()
