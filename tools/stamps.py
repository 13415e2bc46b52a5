"""Per-phase cycle breakdown of the fused kernel from in-kernel s_memtime stamps.

The stamps run in the DIAG instance, or — in a library built with -DCET_C2_STAMPS (tools/session.sh
builds it as libcet_c2st.so) — in the C2 production instance the bench times.  Phase durations are
s_memtime differences inside one workgroup; workgroup start / end offsets come from s_memrealtime
(the constant 100 MHz clock, comparable across workgroups and XCDs — s_memtime is not).

Usage (GPU box): python tools/stamps.py [B] > gpurun_out/stamps.txt
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from channelestimationtransformer_amd.dataset import make_batch  # noqa: E402

def names(e_layers=(4,), d_layers=3):
    """Phase names in STAMP order: per encoder its embedding, layers (attention, O-proj + LN1, FFN + LN2, distil
    conv on all but the last) and norm; then the decoder."""
    n = ["start"]
    for e, nl in enumerate(e_layers):
        p = f"E{e} " if len(e_layers) > 1 else ""
        n += [f"{p}embedding"]
        n += sum([[f"{p}L{l} attention", f"{p}L{l} O-proj+LN1", f"{p}L{l} FFN+LN2"] +
                  ([f"{p}L{l} conv+pool"] if l < nl - 1 else []) for l in range(nl)], [])
        n += [f"{p}enc norm"]
    n += ["dec embedding"] + sum([[f"D{l} self-attn", f"D{l} cross-attn", f"D{l} O/LN/FFN rest"]
                                  for l in range(d_layers)], []) + ["final norm+proj"]
    return n


NAMES = names()


def stragglers(sub, start, end, tot, clk):
    """Where the last workgroups ran (slots 96 / 97: HW_ID and XCC_ID, gfx9 field layout): end-time tail,
    per-XCC ends, workgroups per CU, and what the latest 5 % have in common."""
    hw, xcc = sub[:, 96].astype(np.int64), sub[:, 97].astype(np.int64)
    if not hw.any():
        return
    xcc = xcc & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    simd = (hw >> 4) & 3
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    q = np.percentile(end, [50, 90, 99])
    print(f"WG end tail: p50 {q[0]:.2f}  p90 {q[1]:.2f}  p99 {q[2]:.2f}  max {end.max():.2f} us")
    for x in np.unique(xcc):
        m = xcc == x
        print(f"  XCC {x}: {m.sum()} WGs, {len(np.unique(key[m]))} CUs, end median {np.median(end[m]):.2f} max "
              f"{end[m].max():.2f} us, clock median {np.median(clk[m]):.3f} GHz, WG cycles median {np.median(tot[m]):.0f}")
    ukeys, counts = np.unique(key, return_counts=True)
    hist = {int(c): int((counts == c).sum()) for c in np.unique(counts)}
    print(f"  CUs used {len(ukeys)}; WGs per CU: {hist}")
    per_cu = {k: c for k, c in zip(ukeys, counts)}
    late = end >= np.percentile(end, 95)
    wpc = np.array([per_cu[k] for k in key])
    print(f"  latest 5 %: start offset mean {start[late].mean():.2f} us (all {start.mean():.2f}), WG cycles mean "
          f"{tot[late].mean():.0f} (all {tot.mean():.0f}), clock mean {clk[late].mean():.3f} GHz (all {clk.mean():.3f}), "
          f"WGs on their CU mean {wpc[late].mean():.2f} (all {wpc.mean():.2f}), first SIMD of wave 0: "
          f"{np.bincount(simd[late], minlength=4).tolist()}")
    # a CU's two workgroups: the later one's end against the earlier one's
    bidx = np.arange(len(key))   # v4: every workgroup stamps its own row, so the row is the block index
    two = [np.nonzero(key == k)[0] for k in ukeys if per_cu[k] == 2]
    if two:
        dif = np.array([bidx[i[1]] - bidx[i[0]] for i in two])
        vals, cnts = np.unique(dif, return_counts=True)
        first_low = np.mean([end[i[0]] <= end[i[1]] for i in two])
        print(f"  CU pair block-index distance (top): " +
              ", ".join(f"{v}: {c}" for v, c in sorted(zip(vals, cnts), key=lambda t: -t[1])[:4]) +
              f";  the lower block index ends first in {100 * first_low:.0f} % of pairs")
    pairs = [np.sort(end[key == k]) for k in ukeys if per_cu[k] == 2]
    if pairs:
        pe = np.array(pairs)
        print(f"  CU pairs: first end median {np.median(pe[:, 0]):.2f}, second end median {np.median(pe[:, 1]):.2f}, "
              f"gap median {np.median(pe[:, 1] - pe[:, 0]):.2f} p90 {np.percentile(pe[:, 1] - pe[:, 0], 90):.2f} us")


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    e43 = len(sys.argv) > 2 and sys.argv[2] == "e43"   # the TimingAnalysis stack (attn full, e_layers [4, 3])
    dev = torch.device("cuda:0")
    if e43:
        from channelestimationtransformer_amd.latency import CONFIG, build

        m = build(dict(CONFIG), dev)
        global NAMES
        NAMES = names((4, 3))
    else:
        m = bench.build_model(dev)
    eng = m.engine(dev)
    eng.seed(1)
    xe, xd, _ = make_batch(B, seed=5)
    xe = torch.from_numpy(xe).to(dev)
    xd = torch.from_numpy(xd).to(dev)
    out = torch.empty(B, 5, 16, device=dev)
    for _ in range(10):
        eng.forward(xe, xd, out)
    st = torch.zeros(B * 128, dtype=torch.int64, device=dev)
    eng.set_stamps(st)
    eng.forward(xe, xd, out)
    torch.cuda.synchronize()
    eng.set_stamps(None)
    s = st.view(B, 128).cpu().numpy().astype(np.int64)
    rows = s[:, 0] != 0        # v5 stamps each workgroup (two sequences) in its first sequence's row
    s = s[rows]
    print(f"kernel path: {eng.last_path()}  instance: {eng.last_kernel()}  stamped workgroups: {int(rows.sum())}")
    n = len(NAMES)
    s = s[:, :n]
    d = np.diff(s, axis=1)
    tot = s[:, -1] - s[:, 0]
    print(f"B={B}  per-WG total cycles: mean {tot.mean():.0f}  min {tot.min()}  max {tot.max()}")
    sub = st.view(B, 128).cpu().numpy().astype(np.int64)[rows]
    rt0, rt1 = sub[:, 98], sub[:, 99]
    if rt0.all() and rt1.all():
        # s_memrealtime: 100 MHz, one clock for the whole chip
        span = (rt1.max() - rt0.min()) / 100.0
        start, end = (rt0 - rt0.min()) / 100.0, (rt1 - rt0.min()) / 100.0
        clk = (s[:, -1] - sub[:, 127]) / ((rt1 - rt0) / 100.0) / 1e3   # GHz: s_memtime ticks per realtime us
        print(f"kernel span (first WG start -> last WG end): {span:.2f} us;  WG start offsets: median "
              f"{np.median(start):.2f} us, max {start.max():.2f} us;  WG end: median {np.median(end):.2f} us, "
              f"min {end.min():.2f} us;  in-kernel clock (memtime/realtime): median {np.median(clk):.3f} GHz")
        stragglers(sub, start, end, tot, clk)
    SUBN = ["K/V projection", "Q projection", "phase A (M)", "top-u select", "phase C (softmax·V)", "phase D (rest)"]
    for c, base in ((0, 100), (1, 108)):
        ss = sub[:, base:base + 7]
        if not ss.any():
            continue
        dd = np.diff(ss, axis=1)
        print(f"call {c} head 0 sub-phases: " + "  ".join(f"{SUBN[i]} {dd[:, i].mean():.0f}" for i in range(6)))
    # encoder layer 0 fine stamps (slots 116..123) between the phase stamps 2 (attention end) and 5
    f = sub[:, 116:124]
    if f.any():
        pts = np.concatenate([sub[:, 2:3], f[:, 0:1], sub[:, 3:4], f[:, 1:5], f[:, 5:8], sub[:, 5:6]], axis=1)
        lab = ["O-proj gemm", "LN1", "FFN1+GELU", "barrier", "FFN2 gemm", "LN2", "conv gemm", "maxpool",
               "barrier", "store_xb+barrier"]
        dd = np.diff(pts, axis=1).mean(axis=0)
        print("L0 fine: " + "  ".join(f"{a} {b:.0f}" for a, b in zip(lab, dd)))
    # L0 LayerNorms (C2 + stamps build): per wave, s_memtime at LN entry (its own GEMM done), after the partials
    # barrier, after the statistics barrier and at exit, relative to the phase start (slots 32..63 LN1, 64..95 LN2)
    for nm, base, p0, p1 in (("LN1", 32, 2, 3), ("LN2", 64, 3, 4)):
        ln = sub[:, base:base + 32].reshape(-1, 8, 4)
        if not ln.all():
            continue
        rel = (ln - sub[:, p0][:, None, None]).mean(axis=0)
        end = (sub[:, p1] - sub[:, p0]).mean()
        print(f"L0 {nm} per wave (cycles after the phase start; phase ends at {end:.0f}): "
              "entry / after partials barrier / after stats barrier / exit")
        for w in range(8):
            print(f"    wave {w}: {rel[w, 0]:7.0f} {rel[w, 1]:7.0f} {rel[w, 2]:7.0f} {rel[w, 3]:7.0f}")
        ent = ln[:, :, 0]
        print(f"  {nm}: entry skew (last − first wave) mean {(ent.max(1) - ent.min(1)).mean():.0f}; "
              f"last entry → partials barrier released {(ln[:, :, 1].min(1) - ent.max(1)).mean():.0f}; "
              f"stats phase {(ln[:, :, 2].min(1) - ln[:, :, 1].max(1)).mean():.0f}; "
              f"apply {(ln[:, :, 3] - ln[:, :, 2]).mean():.0f}; last exit → phase end "
              f"{(sub[:, p1] - ln[:, :, 3].max(1)).mean():.0f}")
    e = sub[:, 124:128]
    if e[:, 0].any():
        pts = np.stack([e[:, 3], sub[:, 0], e[:, 0], e[:, 1], sub[:, 1]], axis=1)
        dd = np.diff(pts, axis=1).mean(axis=0)
        lab = ["entry+LDS zero", "stage x_enc", "embed gemm+pe", "store+barrier"]
        print("embedding fine: " + "  ".join(f"{a} {b:.0f}" for a, b in zip(lab, dd)))
    for i in range(1, n):
        print(f"{NAMES[i]:22s} mean {d[:, i - 1].mean():9.0f}  p10 {np.percentile(d[:, i - 1], 10):9.0f}  "
              f"p90 {np.percentile(d[:, i - 1], 90):9.0f}  ({100 * d[:, i - 1].mean() / tot.mean():5.1f}%)")


if __name__ == "__main__":
    main()
