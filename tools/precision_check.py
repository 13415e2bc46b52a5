"""Every golden fixture through the v4 kernel at each operand precision: rel-NMSE against the
reference fixture and the oracle, selection agreement, kernel time at B=512 (one JSON line each).

    python tools/precision_check.py
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from engine_util import model_for, run_engine  # noqa: E402
from golden_util import case_names, load_case, oracle_for, rel_nmse  # noqa: E402

dev = torch.device("cuda:0")
for name in [n for n in case_names() if n.startswith("informer")]:
    case = load_case(name)
    for prec in ("bf16", "split-bf16", "fp8"):
        if prec == "fp8" and case.meta["model"] != "informer_lsq":
            continue
        m = model_for(case)
        eng = m.engine(dev)
        try:
            eng.set_precision(prec)
            got = eng.precision()
        except Exception as exc:  # noqa: BLE001
            print(json.dumps({"case": name, "prec": prec, "error": str(exc)}), flush=True)
            continue
        out, dbg, (buf, layout, per) = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx, debug=True,
                                                  attns=True)
        res = {"case": name, "prec": got, "rel_nmse_fixture": rel_nmse(out, case.z["out"])}
        ref, _ = oracle_for(case).forward(case.z["x_enc"], case.z["x_dec"], case.idx)
        res["rel_nmse_oracle"] = rel_nmse(out, ref)
        # selections vs the fixture's M_top (sparse calls)
        flips = 0
        for k in range(case.meta["n_mtop"]):
            mt = case.z[f"mtop{k}"]
            Mk = dbg.get(f"M{k}")
            if Mk is None or not np.isfinite(Mk).all():
                continue
            u = mt.shape[-1]
            sel = np.sort(np.argsort(-Mk, axis=-1, kind="stable")[..., :u], axis=-1)
            flips += int((sel != mt).any(-1).sum())
        res["selection_mismatches"] = flips
        maps = [(k, v) for k, v in case.z.items() if k.startswith("attn_e0_l")]
        if maps:
            errs = []
            for l, (off, L) in enumerate(layout):
                if f"attn_e0_l{l}" in case.z:
                    errs.append(rel_nmse(buf[off:off + 8 * L * L].reshape(8, L, L), case.z[f"attn_e0_l{l}"]))
            res["attn_rel_nmse_max"] = max(errs) if errs else None
        print(json.dumps(res), flush=True)
