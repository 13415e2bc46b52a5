"""Where a short timed region (the driver's --steps 20) loses time against a long one: bench.py's lanes,
timed loops of K steps with host and GPU-side (event) clocks, the host loop's own duration, and the
per-step GPU spans of lane 0.

    python tools/steps_probe.py [K ...]      (GPU box)
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from channelestimationtransformer_amd.dataset import make_batch  # noqa: E402


def main():
    ks = [int(a) for a in sys.argv[1:]] or [20, 300]
    dev = torch.device("cuda:0")
    B, T, NL = 512, 5, 2
    all_sums = torch.zeros(1001, 2, T, dtype=torch.float64, device=dev)
    lanes = []
    for i in range(NL):
        eng = bench.build_model(dev).engine(dev)
        eng.seed(1 + i)
        xe, xd, lab = (torch.from_numpy(a).to(dev) for a in make_batch(B, seed=1234 + 104729 * i))
        out = torch.empty(B, T, 16, device=dev)
        st = torch.cuda.Stream(dev)
        lanes.append(dict(eng=eng, st=st, keep=(xe, xd, lab, out),
                          fused=eng.bind_forward_nmse(xe, xd, out, lab, all_sums, st.cuda_stream)))

    def warm(n=2000):
        for k in range(n):
            lanes[k % NL]["fused"](1000)
        torch.cuda.synchronize(dev)

    def timed(K, events=False, gap_us=0.0, poll=False):
        warm(600)
        if gap_us:
            t = time.perf_counter()
            while (time.perf_counter() - t) * 1e6 < gap_us:
                pass
        ev = [(torch.cuda.Event(enable_timing=events), torch.cuda.Event(enable_timing=events)) for _ in range(NL)]
        t0 = time.perf_counter()
        if events:
            for i in range(NL):
                ev[i][0].record(lanes[i]["st"])
        for k in range(K):
            lanes[k % NL]["fused"](k)
        t_loop = time.perf_counter() - t0
        if events or poll:
            for i in range(NL):
                ev[i][1].record(lanes[i]["st"])
        if poll:   # busy-poll the lanes' end events (no blocking wait), then the synchronize returns at once
            for i in range(NL):
                while not ev[i][1].query():
                    pass
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        g = [ev[i][0].elapsed_time(ev[i][1]) for i in range(NL)] if events else None
        return dt, t_loop, g

    for K in ks:
        for label, kw in (("plain", {}), ("events", {"events": True}), ("poll", {"poll": True}),
                          ("plain", {}), ("poll", {"poll": True})):
            rs = [timed(K, **kw) for _ in range(5)]
            dts = sorted(r[0] for r in rs)
            loops = sorted(r[1] for r in rs)
            line = (f"K={K:4d} {label:16s} ms/step host median {dts[2] / K * 1e3:.4f} (min {dts[0] / K * 1e3:.4f})  "
                    f"host loop {loops[2] * 1e3:.3f} ms")
            if rs[0][2]:
                line += "  GPU spans per lane ms " + " ".join(f"{x:.3f}" for x in rs[2][2])
            print(line, flush=True)


if __name__ == "__main__":
    main()
