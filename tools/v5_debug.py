"""v5 vs v4 per-sequence comparison (GPU box): for several fixture models and batch sizes, the relative
difference of each sequence's output between the generations, split by v5 slot (even / odd index), and
each generation against the float64 oracle on a few rows.
python tools/v5_debug.py > gpurun_out/v5_debug.txt"""
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


def per_seq(a, b):
    return ((a - b) ** 2).sum((1, 2)) / (b ** 2).sum((1, 2))


def main():
    dev = torch.device("cuda:0")
    cases = [("informer_prob_e43", 2), ("informer_prob_e43", 64), ("informer_full_e43", 600),
             ("informer_single_e3", 64), ("informer_prob_seq48", 64), ("informer_prob_b4", 64)]
    if os.environ.get("V5_CASES"):
        cases = [(c.split(":")[0], int(c.split(":")[1])) for c in os.environ["V5_CASES"].split(",")]
    for name, B in cases:
        case = load_case(name)
        m = model_for(case)
        cfg = case.cfg
        eng = m.engine(dev)
        xe, xd, _ = make_batch(B, cfg["seq_len"], cfg["label_len"], cfg["pred_len"], seed=3000 + B)
        outs = {}
        for v in (5, 4):
            eng.set_variant(v)
            outs[v], _, _ = run_engine(m, xe, xd, case.idx)
            outs[f"p{v}"] = eng.last_path()
        eng.set_variant(5)
        d = per_seq(outs[5], outs[4])
        rows = np.arange(min(B, 4))
        ref, _ = oracle_for(case).forward(xe[rows], xd[rows], case.idx)
        e5, e4 = per_seq(outs[5][rows], ref), per_seq(outs[4][rows], ref)
        print(f"{name} B={B} paths={outs['p5']},{outs['p4']}  v5-v4 per-seq: even max {d[0::2].max():.2e} "
              f"odd max {d[1::2].max():.2e} n>1e-8 {(d > 1e-8).sum()}  vs oracle rows {list(rows)}: "
              f"v5 {np.array2string(e5, precision=2)} v4 {np.array2string(e4, precision=2)}", flush=True)


if __name__ == "__main__":
    main()
