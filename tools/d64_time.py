"""Launch time of the d_model-64 checkpoint architecture's forward (seq_len 25, e_layers [4,3], attn "full";
the fused layer-wise form) at batch B: back-to-back launches between two HIP events, and the output's
checksum so builds can be compared for equality.

    python tools/d64_time.py [B] [launches] [precision]      (GPU box; CET_LIB selects the build)
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from bench_configs import informer  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
N = int(sys.argv[2]) if len(sys.argv) > 2 else 200
dev = torch.device("cuda:0")
m, _ = informer(dev, [4, 3], "full", seq_len=25, d_model=64)
eng = m.engine(dev)
if len(sys.argv) > 3:   # e.g. "bf16": the bf16-operand instance of the fused form
    eng.set_precision(sys.argv[3])
g = torch.Generator().manual_seed(5)
xe = torch.randn(B, 25, 16, generator=g).to(dev)
xd = torch.randn(B, 15, 16, generator=g).to(dev)
out = torch.empty(B, 5, 16, device=dev)
for _ in range(20):
    eng.forward(xe, xd, out)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(N):
    eng.forward(xe, xd, out)
ev1.record()
torch.cuda.synchronize()
ms = ev0.elapsed_time(ev1) / N
print(f"path {eng.last_path()}  B {B}  ms per launch {ms:.4f}  seq/s {B / ms * 1e3:.0f}  "
      f"checksum {float(out.double().sum()):.10e}", flush=True)
