"""Per-stage parity report of the HIP engine against the CPU oracle for every fixture case.

Usage (GPU box):  python tools/parity_report.py [case ...]  > gpurun_out/parity.txt
"""
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

from golden_util import case_names, load_case, rel_nmse  # noqa: E402
from engine_util import model_for, run_engine, stage_report  # noqa: E402


def main(names):
    for name in names or case_names():
        case = load_case(name)
        print(f"== {name}  B={case.meta['B']}", flush=True)
        try:
            m = model_for(case)
            out, dbg, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx, debug=True)
            rep, ref, trace = stage_report(case, out, dbg)
            print(f"   out vs reference fixture: rel-NMSE {rel_nmse(out, case.z['out']):.3e}")
            for k, v in rep.items():
                print(f"   {k:14s} {v:.3e}")
            for k, mt in enumerate(trace.m_top):
                if f"M{k}" in dbg:
                    Mk = dbg[f"M{k}"]
                    u = mt.shape[-1]
                    sel = np.sort(np.argsort(-Mk, axis=-1, kind="stable")[..., :u], axis=-1)
                    flips = int((sel != mt).any(-1).sum())
                    print(f"   M_top call {k}: (b,h) rows with a different selection: {flips}/{mt.shape[0] * mt.shape[1]}")
        except Exception:
            traceback.print_exc()
            sys.stdout.flush()


if __name__ == "__main__":
    main(sys.argv[1:])
