"""Static check of vector-memory load completion in gfx950 assembly: every VGPR read must come after an
`s_waitcnt vmcnt(N)` that retires the load writing it, on EVERY path through the control flow.

Model (MI355X_MICROARCH "s_waitcnt vmcnt(N)"): loads, stores and atomics of the vector memory path count
together in issue order; vmcnt(N) waits until all but the N youngest are done.  The scan runs a forward
dataflow over the kernel's basic blocks; the state is the queue of outstanding operations (youngest first),
each with the VGPRs it will write, and a join keeps, position by position, the union of the incoming queues
(longest length), so a register still in flight on any incoming path stays in flight.  A read (or a write)
of a register that may still be in flight is reported with the instruction and the load that wrote it.

    python tools/vmcnt_scan.py file.s [kernel-substring] [max-reports]
"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
BR = re.compile(r"^s_(cbranch_\w+|branch)\s+(\S+)")
VMEM = ("buffer_load", "global_load", "scratch_load", "flat_load", "buffer_store", "global_store", "scratch_store",
        "flat_store", "buffer_atomic", "global_atomic", "flat_atomic")


def vregs(tok):
    out = set()
    for m in REG.finditer(tok):
        if m.group(1) is not None:
            out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def parse(lines, want):
    """[(label|None, [(op, operands, lineno)])] basic blocks of the first kernel whose name contains `want`."""
    blocks, cur, inside = [], None, False
    for i, ln in enumerate(lines):
        s = ln.split(";")[0].strip()
        if not inside:
            if s.endswith(":") and s[:-1].startswith("_Z") and (want is None or want in s):
                inside = True
                cur = (None, [])
                blocks.append(cur)
            continue
        if s.endswith(":"):
            cur = (s[:-1], [])
            blocks.append(cur)
            continue
        if not s or s.startswith("."):
            continue
        op = s.split()[0]
        cur[1].append((op, s[len(op):].strip(), i + 1))
        if op == "s_endpgm":
            break
        if BR.match(s):   # a branch ends its basic block: what follows is the fall-through block
            cur = (None, [])
            blocks.append(cur)
    return blocks


def successors(blocks):
    idx = {lab: k for k, (lab, _) in enumerate(blocks) if lab}
    succ = []
    for k, (_, ins) in enumerate(blocks):
        s = []
        last = ins[-1] if ins else None
        fall = True
        for op, args, _ in ins:
            m = BR.match(f"{op} {args}")
            if m:
                tgt = args.split()[0]
                if tgt in idx:
                    s.append(idx[tgt])
                if op == "s_branch":
                    fall = False
            if op in ("s_endpgm", "s_setpc_b64"):
                fall = False
        if fall and k + 1 < len(blocks) and not (last and last[0] == "s_endpgm"):
            s.append(k + 1)
        succ.append(s)
    return succ


def step(state, op, args, line, report):
    """Apply one instruction to the queue (tuple of (frozenset(regs), line) youngest first)."""
    q = list(state)
    if op == "s_waitcnt":
        m = re.search(r"vmcnt\((\d+)\)", args)
        if m:
            q = q[:int(m.group(1))]
        return tuple(q)
    parts = [p.strip() for p in args.split(",")]
    is_vmem = op.startswith(VMEM)
    dst, srcs = set(), set()
    if parts and parts[0]:
        if is_vmem and ("store" in op or ("atomic" in op and "glc" not in args and " sc0" not in args)):
            srcs = vregs(",".join(parts))
        elif op.startswith(("v_", "buffer_load", "global_load", "scratch_load", "flat_load", "ds_", "buffer_atomic",
                            "global_atomic", "flat_atomic")):
            dst = vregs(parts[0])
            srcs = vregs(",".join(parts[1:]))
        else:
            srcs = vregs(",".join(parts))
    inflight = {}
    for regs, ln in q:
        for r in regs:
            inflight.setdefault(r, ln)
    # a VMEM load may overwrite the destination of an older one in flight (they return in issue order);
    # every other write, and every read, of an in-flight register is a hazard
    for r in sorted((srcs | (set() if is_vmem else dst)) & set(inflight)):
        report.add((line, op, r, inflight[r]))
    if is_vmem:
        q.insert(0, (frozenset(dst) if dst else frozenset(), line))
        q = q[:64]   # vmcnt saturates at 63 outstanding operations
    return tuple(q)


def scan(path, want=None):
    lines = open(path, errors="replace").read().split("\n")
    blocks = parse(lines, want)
    succ = successors(blocks)
    # the state per block entry: tuple of frozensets of (reg) tagged by load line; kept as tuple of (regs, line)
    entry = [None] * len(blocks)
    entry[0] = ()
    work = [0]
    report = set()
    seen = 0
    while work:
        k = work.pop()
        seen += 1
        st = entry[k]
        for op, args, line in blocks[k][1]:
            st = step(st, op, args, line, report)
        for s in succ[k]:
            new = merge(entry[s], st)
            if new != entry[s]:
                entry[s] = new
                work.append(s)
    return blocks, report


def merge(a, b):
    """Join of two queues of (regs, line): position-wise union (a register's earliest load line kept)."""
    if a is None:
        return b
    n = max(len(a), len(b))
    out = []
    for i in range(n):
        ra, la = a[i] if i < len(a) else (frozenset(), 10 ** 9)
        rb, lb = b[i] if i < len(b) else (frozenset(), 10 ** 9)
        out.append((ra | rb, min(la, lb)))
    return tuple(out)


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else None
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    blocks, report = scan(path, want)
    n_ins = sum(len(b[1]) for b in blocks)
    print(f"{len(blocks)} blocks, {n_ins} instructions, {len(report)} reads/writes of registers possibly in flight")
    for line, op, r, ld in sorted(report)[:top]:
        print(f"  line {line}: {op} uses v{r} (VMEM op at line {ld} may still be in flight)")


if __name__ == "__main__":
    main()
