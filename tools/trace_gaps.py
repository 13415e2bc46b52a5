"""Inter-dispatch gaps of back-to-back kernels from a rocprofv3 --kernel-trace rocpd database:
python tools/trace_gaps.py run_results.db [kernel-substring]"""
import sqlite3
import sys

import numpy as np


def main():
    db = sqlite3.connect(sys.argv[1])
    sub = sys.argv[2] if len(sys.argv) > 2 else "informer_forward"
    cur = db.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    suf = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch_"))[len("rocpd_kernel_dispatch_"):]
    rows = cur.execute(f"select d.start, d.end, k.display_name from rocpd_kernel_dispatch_{suf} d "
                       f"join rocpd_info_kernel_symbol_{suf} k on d.kernel_id = k.id order by d.start").fetchall()
    names = sorted({r[2] for r in rows})
    for n in names:
        print("kernel:", n[:110], sum(1 for r in rows if r[2] == n))
    ks = [r for r in rows if sub in r[2]]
    st = np.array([r[0] for r in ks], dtype=np.float64)
    en = np.array([r[1] for r in ks], dtype=np.float64)
    dur = (en - st) / 1e3
    gap = (st[1:] - en[:-1]) / 1e3
    per = (st[1:] - st[:-1]) / 1e3
    # the timed run is the last 20 launches (bench.py --steps 20 after warm-up)
    tail = slice(-20, None)
    print(f"{len(ks)} dispatches of *{sub}*; last 20: kernel {np.median(dur[tail]):.2f} us median "
          f"({dur[tail].mean():.2f} mean); gap end->start {np.median(gap[-19:]):.2f} us median "
          f"({gap[-19:].mean():.2f} mean, max {gap[-19:].max():.2f}); start->start {np.median(per[-19:]):.2f} us")
    others = [r for r in rows if sub not in r[2] and r[0] >= ks[-20][0]]
    print(f"other dispatches inside the last 20 steps: {len(others)}")


if __name__ == "__main__":
    main()
