"""Scan a gfx950 assembly file for MFMA → VALU read-after-write distances, split by whether an inline-asm
block (;;#ASMSTART) sits between the MFMA and the first VALU that reads its result.  The hazard recognizer
counts wait states by instruction; if it credits an EMPTY inline asm as a wait state, the distances with
asm in between come out shorter than the minimum the compiler keeps elsewhere.
python tools/mfma_hazard_scan.py file.s [kernel-substring]"""
import re
import sys
from collections import Counter


def regs(tok):
    """v[a:b] / vN / a[..] → set of (kind, index)."""
    out = set()
    for m in re.finditer(r"\b([va])\[(\d+):(\d+)\]", tok):
        k, a, b = m.group(1), int(m.group(2)), int(m.group(3))
        out |= {(k, i) for i in range(a, b + 1)}
    for m in re.finditer(r"\b([va])(\d+)\b", tok):
        out.add((m.group(1), int(m.group(2))))
    return out


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else None
    lines = open(path).read().split("\n")
    insts = []   # (op, dst_regs, src_regs, is_asm_marker, lineno)
    cur = None
    for i, ln in enumerate(lines):
        s = ln.split(";")[0].strip() if not ln.strip().startswith(";;#ASM") else ln.strip()
        if s.endswith(":") and s[:-1].startswith("_Z"):
            cur = s[:-1]
            continue
        if want and (cur is None or want not in cur):
            continue
        if s.startswith(";;#ASMSTART"):
            insts.append(("ASM", set(), set(), True, i, s))
            continue
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        op = s.split()[0]
        rest = s[len(op):]
        parts = [p.strip() for p in rest.split(",")]
        dst = regs(parts[0]) if parts and parts[0] else set()
        src = set()
        for p in parts[1:]:
            src |= regs(p)
        insts.append((op, dst, src, False, i, s))
    gaps = {False: Counter(), True: Counter()}
    worst = []
    for k, (op, dst, src, _, ln, _t) in enumerate(insts):
        if "mfma" not in op:
            continue
        ws, asm = 0, False
        for op2, d2, s2, is_asm, ln2, t2 in insts[k + 1:k + 40]:
            if is_asm:
                asm = True
                continue
            if op2.startswith("v_") and "mfma" not in op2 and (s2 & dst):
                gaps[asm][ws] += 1
                if asm:
                    worst.append((ws, ln + 1, ln2 + 1, op, op2))
                break
            if op2 == "s_nop":
                ws += int(t2.split()[1]) + 1
            else:
                ws += 1
    for asm in (False, True):
        print(("with inline asm between" if asm else "no asm between"), "wait-state histogram:",
              dict(sorted(gaps[asm].items())))
    worst.sort()
    for w in worst[:15]:
        print("asm case:", w)


if __name__ == "__main__":
    main()
