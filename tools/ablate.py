"""Kernel-time ablations of the fused Informer (C2, B=512): kernel variant × ProbSparse draw source.

  resident : the kernel replays torch's mt19937 stream itself (production path, cet_mt.hpp)
  host     : host-built multiplicity tables staged per forward (no replay inside the kernel)

python tools/ablate.py [variants...]   → one line per (variant, mode): mean kernel µs per launch
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from channelestimationtransformer_amd.dataset import make_batch  # noqa: E402
from channelestimationtransformer_amd.rng import draw_indices  # noqa: E402
from oracle.informer_np import InformerConfig, sample_shapes  # noqa: E402


def run(eng, xe, xd, out, host_idx, n=100):
    for i in range(n + 10):
        if host_idx is not None:
            eng.set_indices(host_idx)
        if i == 10:
            torch.cuda.synchronize()
            eng.timing(True)
        eng.forward(xe, xd, out)
    torch.cuda.synchronize()
    ms, k = eng.timing_read()
    eng.timing(False)
    return 1e3 * ms / max(k, 1)


def main():
    variants = [int(v) for v in sys.argv[1:]] or [4]
    dev = torch.device("cuda:0")
    m = bench.build_model(dev)
    eng = m.engine(dev)
    B = 512
    xe, xd, _ = make_batch(B, seed=5)
    xe, xd = torch.from_numpy(xe).to(dev), torch.from_numpy(xd).to(dev)
    out = torch.empty(B, 5, 16, device=dev)
    idx = draw_indices(sample_shapes(InformerConfig()), seed=3)
    for v in variants:
        eng.set_variant(v)
        eng.seed(1)
        t_res = run(eng, xe, xd, out, None)
        eng.set_sampler(True)
        t_nh = run(eng, xe, xd, out, None)
        eng.set_sampler(False)
        t_host = run(eng, xe, xd, out, idx)
        eng.seed(1)
        t_res2 = run(eng, xe, xd, out, None)
        print(f"variant {v}: resident sampler again {t_res2:8.1f} us", flush=True)
        print(f"variant {v}: resident sampler {t_res:8.1f} us   native host sampler {t_nh:8.1f} us   "
              f"host tables {t_host:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
