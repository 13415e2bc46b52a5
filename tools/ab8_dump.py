"""Round-5 diagnostic of the round-4 ab8 candidate: the first 6-tile attention call of workgroup 0, head 0, in the
split-bf16 production instance against the diagnostic instance on the same inputs (fixture informer_full_e43).
Needs a library built with -DCET_AB8_DUMP (cet_ab8_dump).  Prints which dumped quantity first differs."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from channelestimationtransformer_amd._lib import lib  # noqa: E402
from engine_util import model_for, run_engine  # noqa: E402
from golden_util import load_case  # noqa: E402

lib.cet_ab8_dump.restype = ctypes.c_int
lib.cet_ab8_dump.argtypes = [ctypes.c_void_p, ctypes.c_int]



def dump(debug):
    case = load_case(sys.argv[1] if len(sys.argv) > 1 else "informer_full_e43")
    m = model_for(case)
    m.engine(torch.device("cuda:0")).set_precision("split-bf16")
    lib.cet_ab8_dump(None, 1)
    out, _, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx, debug=debug)
    torch.cuda.synchronize()
    buf = (ctypes.c_uint * (8 * 128 * 64))()
    lib.cet_ab8_dump(buf, 0)
    return out, np.frombuffer(buf, dtype=np.uint32).reshape(8, 128, 64).copy(), m.engine(torch.device("cuda:0")).last_kernel()


prod, dp, kp = dump(False)
diag, dd, kd = dump(True)
print("production:", kp, " diag:", kd, " outputs equal:", np.array_equal(prod, diag),
      " max |diff|:", float(np.abs(prod - diag).max()))
names = {}
for t in range(6):
    names[4 * t] = names[4 * t + 1] = f"K tile {t} hi"
    names[4 * t + 2] = names[4 * t + 3] = f"V tile {t} hi"
    names[24 + 4 * t] = names[24 + 4 * t + 1] = f"K tile {t} lo"
    names[24 + 4 * t + 2] = names[24 + 4 * t + 3] = f"V tile {t} lo"
names.update({48: "q hi", 49: "q hi", 50: "score max", 51: "exp sum", 52: "o", 53: "o", 54: "o", 55: "o",
              56: "q lo", 57: "q lo", 127: "written"})
for st in range(6):
    for j, nm in enumerate(["max", "sum", "o0", "o1", "o2", "o3", "query"]):
        names[64 + 8 * st + j] = f"tile {st} {nm}"
for h in range(8):
    bad = []
    for r in range(128):
        if r in names and not np.array_equal(dp[h, r], dd[h, r]):
            lanes = np.nonzero(dp[h, r] != dd[h, r])[0]
            bad.append(f"{names[r]} ({len(lanes)} lanes, lane {lanes[0]}: 0x{dp[h, r][lanes[0]]:08x} vs 0x{dd[h, r][lanes[0]]:08x})")
    print(f"head {h}: " + ("all equal" if not bad else "; ".join(bad[:6])))
