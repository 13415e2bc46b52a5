"""Per-stage, per-sequence parity of the fused kernel's activation dumps against the float64 oracle
(GPU box): python tools/v5_stages.py [case] [B] [variant]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from channelestimationtransformer_amd.dataset import make_batch  # noqa: E402
from engine_util import model_for, run_engine  # noqa: E402
from golden_util import load_case, oracle_for  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "informer_prob_e43"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    variant = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    case = load_case(name)
    m = model_for(case)
    cfg = case.cfg
    eng = m.engine(torch.device("cuda:0"))
    eng.set_variant(variant)
    xe, xd, _ = make_batch(B, cfg["seq_len"], cfg["label_len"], cfg["pred_len"], seed=77)
    out, dbg, _ = run_engine(m, xe, xd, case.idx, debug=True)
    acts = {}
    ref, _ = oracle_for(case).forward(xe, xd, case.idx, acts=acts)
    print(f"{name} B={B} path={eng.last_path()}")
    for k, v in dbg.items():
        if k not in acts:
            continue
        r = np.asarray(acts[k])
        e = ((v - r) ** 2).sum(axis=tuple(range(1, v.ndim))) / (r ** 2).sum(axis=tuple(range(1, r.ndim)))
        print(f"  {k:16s} " + " ".join(f"{x:.1e}" for x in e[:8]))
    e = ((out - ref) ** 2).sum((1, 2)) / (ref ** 2).sum((1, 2))
    print(f"  {'out':16s} " + " ".join(f"{x:.1e}" for x in e[:8]))


if __name__ == "__main__":
    main()
