"""Per-category cycles of the fused layer-wise kernel (workgroup 0), from the diagnostic build:

    make -C channelestimationtransformer_amd/csrc OUT=../libcet_stamps.so B=build_st EXTRA=-DLWF_STAMPS
    CET_LIB=channelestimationtransformer_amd/libcet_stamps.so python tools/lwf_stamps.py [B] [precision]

Runs the d_model-64 checkpoint architecture (seq_len 25, e_layers [4,3], attn "full") three times at batch B;
the kernel prints one line per launch (GEMM / attention / LayerNorm / other cycles of workgroup 0).
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from bench_configs import informer  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda:0")
m, _ = informer(dev, [4, 3], "full", seq_len=25, d_model=64)
eng = m.engine(dev)
if len(sys.argv) > 2:   # "bf16": the bf16-operand instance
    eng.set_precision(sys.argv[2])
xe = torch.randn(B, 25, 16, device=dev)
xd = torch.randn(B, 15, 16, device=dev)
out = torch.empty(B, 5, 16, device=dev)
for _ in range(3):
    eng.forward(xe, xd, out)
    torch.cuda.synchronize()
print("path", eng.last_path(), flush=True)
