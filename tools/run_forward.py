"""Minimal driver for profilers: N forwards of the C2 Informer at batch B with kernel variant V.

python tools/run_forward.py [N] [B] [V]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from channelestimationtransformer_amd.dataset import make_batch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = int(sys.argv[2]) if len(sys.argv) > 2 else 512
V = int(sys.argv[3]) if len(sys.argv) > 3 else 4
dev = torch.device("cuda:0")
m = bench.build_model(dev)
eng = m.engine(dev)
eng.set_variant(V)
eng.seed(1)
xe, xd, _ = make_batch(B, seed=5)
xe, xd = torch.from_numpy(xe).to(dev), torch.from_numpy(xd).to(dev)
out = torch.empty(B, 5, 16, device=dev)
for _ in range(n):
    eng.forward(xe, xd, out)
torch.cuda.synchronize()
