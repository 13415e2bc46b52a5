"""How often the mixed policy's decoder selections differ from split bf16's (the fp32-level selection) on a
B = 512 batch of the lab20 model (label_len 20: a genuinely sparse masked decoder), and the two outputs' distance
from the float64 oracle on row slices.  The DIAG instances dump every call's M; the top-u sets are rebuilt from
them with the kernel's rank rule.

    python tools/lab20_mixed.py [B]      (GPU box) → one JSON line
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from engine_util import run_engine

    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.informer import InformerStack
    from channelestimationtransformer_amd.rng import draw_indices
    from channelestimationtransformer_amd.weights import synthetic_state_dict
    from oracle.informer_np import InformerConfig, InformerOracle, sample_shapes

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    dev = torch.device("cuda:0")
    m = InformerStack(16, 16, 16, 90, 20, 5, 5, 128, 8, [4], 3, 64, 0.05, "prob", "fixed", "gelu", False, True, dev)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(m._schema(), 3).items()})
    m.eval()
    cfg = InformerConfig(label_len=20)
    idx = draw_indices(sample_shapes(cfg), seed=9)
    xe, xd, _ = make_batch(B, 90, 20, 5, seed=77)
    res = {}
    for prec in ("split-bf16", "mixed"):
        eng = m.engine(dev)
        eng.set_precision(prec)
        out, dbg, _ = run_engine(m, xe, xd, idx, debug=True)
        prod, _, _ = run_engine(m, xe, xd, idx)
        res[prec] = (out, dbg, prod, eng.last_kernel())
    u = [c[1] for c in sample_shapes(cfg)]
    n_calls = len(u)
    lq = [s[0] for s in sample_shapes(cfg)]
    report = {"B": B}
    for k in range(n_calls):
        up = 5 * int(np.ceil(np.log(lq[k])))
        up = min(up, lq[k])
        if up >= lq[k]:
            continue
        sets = {}
        for prec in res:
            Mk = res[prec][1][f"M{k}"]
            sets[prec] = np.sort(np.argsort(-Mk, axis=-1, kind="stable")[..., :up], axis=-1)
        report[f"call{k}_rows_differing"] = int((sets["mixed"] != sets["split-bf16"]).any(-1).sum())
        report[f"call{k}_rows"] = int(np.prod(sets["mixed"].shape[:-1]))
    state = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    rows = np.r_[0:16, B - 16:B]
    ref, _ = InformerOracle(cfg, state).forward(xe[rows], xd[rows], idx)
    for prec in res:
        o = res[prec][2][rows].astype(np.float64)
        report[f"{prec}_rel_nmse_vs_oracle"] = float(np.sum((o - ref) ** 2) / np.sum(ref ** 2))
        report[f"{prec}_kernel"] = res[prec][3]
    print(json.dumps(report))


if __name__ == "__main__":
    main()
