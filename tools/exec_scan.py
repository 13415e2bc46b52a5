"""Build guard: no cross-lane permute/swap issued under a narrowed EXEC in the shipped gfx950 code.

The v4 kernels and the fused layer-wise form reduce across lanes with gfx950's v_permlane16_swap /
v_permlane32_swap (cet_device.hpp xor_sum / xor_max).  Every source-level call sits at full EXEC (the
branches around them are wave-uniform), and a butterfly is only right if every lane took part: a
swap the compiler sinks into an EXEC-narrowed region reads partner lanes whose operand was never
computed.  Bisecting v5 found exactly that (cet_v5.hpp bp_sum; profiles/r03/bisect_*.txt), so this scan
checks the compiled code objects of libcet.so rather than trusting the compiler:

* the code objects are extracted from the library (llvm-objdump --offloading) and disassembled;
* the SI control-flow lowering narrows EXEC for an if / else arm or a divergent loop body and widens it
  again from a mask it kept in an SGPR pair: `s_*_saveexec_b64 sX` (EXEC saved in sX), the else-switch
  (`s_xor_b64 sX, exec, sX`, `s_or_saveexec_b64` / `s_andn2_saveexec_b64` + `s_xor_b64 exec, exec, sY`),
  a loop's exit mask (`s_andn2_b64 exec, exec, sX`, grown by `s_or_b64 sX, .., sX`) and plain copies
  (`s_mov_b64 sX, exec`), each restored by `s_or_b64 exec, exec, sX` / `s_mov_b64 exec, sX`.  A forward
  dataflow over each function's control-flow graph keeps the set of narrowings in force and, per pair,
  the set a restore from it returns to; `v_cmpx`, `s_and_b64 exec, ..` and any EXEC write it cannot
  follow count as narrowing.  A saveexec on a wave-uniform boolean (`s_cselect_b64 sX, -1, 0`, or the
  compiler's `c | ~EXEC` merge around an inner region) is a uniform branch, not a narrowing;
* every v_permlane*_swap / v_permlane*_b32 reached with a narrowing in force is a finding.
Limits: masks spilled to VGPR lanes (v_writelane / v_readlane) are not followed, so a swap behind such a
restore is reported (conservative); the lowering's own conventions are trusted, not a lane-exact model.

    python tools/exec_scan.py [libcet.so] [kernel-substring ...]
Exit status 1 if any finding.  tests/test_isa_guard.py runs it in the CPU suite.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
CROSS_LANE = re.compile(r"^v_permlane(16|32)_swap|^v_permlane(16|x16)_b32")
FN = re.compile(r"^[0-9a-f]+ <(.+)>:$")
ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")


def disassemble(lib: str) -> list[str]:
    """Disassembly text of every gfx950 code object bundled in `lib`."""
    out = []
    with tempfile.TemporaryDirectory() as d:
        so = os.path.join(d, "lib.so")
        shutil.copy(lib, so)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", so], cwd=d, check=True, capture_output=True)
        for f in sorted(os.listdir(d)):
            if "amdgcn" in f and "gfx950" in f and os.path.getsize(os.path.join(d, f)) > 0:
                r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", os.path.join(d, f)],
                                   check=True, capture_output=True, text=True)
                out.append(r.stdout)
    return out


def functions(text: str):
    """(name, [(addr, op, operands)]) per function of one disassembly."""
    name, body = None, []
    for ln in text.split("\n"):
        m = FN.match(ln.strip())
        if m:
            if name:
                yield name, body
            name, body = m.group(1), []
            continue
        if name is None:
            continue
        s = ln.strip()
        a = ADDR.search(s)
        if not s or a is None:
            continue
        ins = s.split("//")[0].strip()
        op = ins.split()[0]
        body.append((int(a.group(1), 16), op, ins[len(op):].strip()))
    if name:
        yield name, body


TERMINATORS = ("s_branch", "s_endpgm", "s_setpc_b64", "s_endpgm_saved")
SAVEEXEC = re.compile(r"^s_(and|andn1|andn2|or|orn1|orn2|xor|nand|nor|xnor)_saveexec_b64$")


def _blocks(body):
    """Basic blocks {start: (end, [successor starts])} of one function."""
    n = len(body)
    addr_ix = {a: i for i, (a, _, _) in enumerate(body)}
    leaders, targets = {0}, {}
    for i, (a, op, ops) in enumerate(body):
        if op == "s_branch" or op.startswith("s_cbranch"):
            tok = ops.split()[0] if ops.split() else ""
            if tok.isdigit():   # SOPP branch: target = next instruction + 4 · simm16
                imm = int(tok)
                t = a + 4 + 4 * (imm - 65536 if imm >= 32768 else imm)
                if t in addr_ix:
                    targets[i] = addr_ix[t]
                    leaders.add(addr_ix[t])
            if i + 1 < n:
                leaders.add(i + 1)
        elif op in TERMINATORS and i + 1 < n:
            leaders.add(i + 1)
    starts = sorted(leaders)
    blocks = {}
    for k, s0 in enumerate(starts):
        e = (starts[k + 1] if k + 1 < len(starts) else n) - 1
        op = body[e][1]
        succ = [targets[e]] if e in targets else []
        if not (op == "s_branch" or op in TERMINATORS) and e + 1 < n:
            succ.append(e + 1)
        blocks[s0] = (e, succ)
    return blocks


def _pairs(tok):
    """SGPR-pair keys a scalar destination writes ('s10' for s[10:11] or s10 or s11)."""
    tok = tok.strip()
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return {f"s{r & ~1}" for r in range(int(m.group(1)), int(m.group(2)) + 1)}
    m = re.fullmatch(r"s(\d+)", tok)
    if m:
        return {f"s{int(m.group(1)) & ~1}"}
    if tok.startswith("vcc"):
        return {"vcc"}
    return set()


def _key(tok):
    k = _pairs(tok)
    return next(iter(k)) if len(k) == 1 and re.fullmatch(r"s\[\d+:\d+\]|vcc", tok.strip()) else None


class St:
    """Dataflow state at one instruction.
    open: tokens of the EXEC narrowings in force (union where paths meet; empty = EXEC as at entry);
    snap: SGPR pair -> the `open` set that restoring EXEC from that pair returns to (a pair saved by an
          s_*_saveexec, copied from EXEC, or holding the lanes a loop exit removed); union of the two
          snapshots where paths meet, dropped if only one path has it;
    ub:   pairs holding a wave-uniform boolean mask (all ones or all zeros);
    orn:  pairs holding such a mask or `uniform boolean | ~EXEC` (both intersections where paths meet)."""
    __slots__ = ("open", "snap", "ub", "orn")

    def __init__(self, open_=frozenset(), snap=None, ub=frozenset(), orn=frozenset()):
        self.open, self.snap, self.ub, self.orn = open_, snap or {}, ub, orn

    def merge(self, o):
        snap = {k: self.snap.get(k, frozenset()) | o.snap.get(k, frozenset()) for k in self.snap.keys() | o.snap.keys()}
        return St(self.open | o.open, snap, self.ub & o.ub, self.orn & o.orn)

    def __eq__(self, o):
        return self.open == o.open and self.snap == o.snap and self.ub == o.ub and self.orn == o.orn


def _step(st, op, ops, addr=0):
    """State after one instruction (the SI control-flow lowering's EXEC algebra, abstracted)."""
    args = [x.strip() for x in ops.split(",")] if ops else []
    open_, snap, ub, orn = st.open, dict(st.snap), st.ub, st.orn
    writes_sgpr = args and (op.startswith("s_") or op.startswith(("v_readlane", "v_readfirstlane", "v_cmp")))
    dst = _pairs(args[0]) if writes_sgpr else set()
    if op.startswith("v_cmp") and op.endswith("_e32"):
        dst = {"vcc"}
    if op.startswith(("v_add_co", "v_sub_co", "v_subrev_co", "v_addc_co", "v_subb_co", "v_div_scale", "v_mad_u64",
                      "v_mad_i64")):
        dst = set().union(*(_pairs(t) for t in args[:2] if not t.startswith("v")))
    tok = ("n", addr)

    def kill(d):
        for k in d:
            snap.pop(k, None)
        return ub - d, orn - d

    if op.startswith("v_cmpx"):
        return St(open_ | {tok}, snap, ub, orn)
    if SAVEEXEC.match(op) and args:
        d, src = args[0], (args[1] if len(args) > 1 else "")
        k, ks = _key(d), _key(src)
        ub2, orn2 = kill(dst)
        if op == "s_and_saveexec_b64":
            if ks in st.orn:   # EXEC ∧ (uniform c [∨ ¬EXEC_inner]): outer EXEC whenever c holds
                new = open_
            else:
                new = open_ | {tok}
            if k:
                snap[k] = open_
            return St(new, snap, ub2, orn2)
        if op in ("s_or_saveexec_b64", "s_andn2_saveexec_b64") and ks in st.snap:
            # else-switch: d = the then lanes; EXEC = the region's outer lanes (or) / its else lanes (andn2)
            outer = st.snap[ks]
            if k:
                snap[k] = outer
            return St(outer if op == "s_or_saveexec_b64" else outer | {tok}, snap, ub2, orn2)
        if k:
            snap[k] = open_
        return St(open_ | {tok}, snap, ub2, orn2)
    if args[:1] == ["exec"]:
        srcs = [x for x in args[1:] if x != "exec"]
        if op == "s_or_b64" and "exec" in args[1:] and srcs and _key(srcs[0]) in st.snap:
            return St(st.snap[_key(srcs[0])] | frozenset(), snap, ub, orn)   # restore: back to the saved state
        if op == "s_or_b64" and "exec" in args[1:]:
            return st   # widening by an unknown mask: stay conservative
        if op == "s_mov_b64" and srcs and _key(srcs[0]) in st.snap:
            return St(st.snap[_key(srcs[0])], snap, ub, orn)
        if op == "s_mov_b64" and srcs and _key(srcs[0]) in st.ub:
            return st
        if op == "s_andn2_b64" and args[1:2] == ["exec"] and len(args) > 2 and _key(args[2]):
            # the removed lanes: EXEC | r restores the state before the first narrowing by r (a loop's
            # later iterations narrow an already narrowed EXEC by the same, grown r)
            snap.setdefault(_key(args[2]), open_)
            return St(open_ | {tok}, snap, ub, orn)
        if op == "s_xor_b64" and args[1:2] == ["exec"] and len(args) > 2 and _key(args[2]) in st.snap:
            return St(open_ | {tok}, snap, ub, orn)   # else arm after s_or_saveexec: d keeps the region
        return St(open_ | {tok}, snap, ub, orn)
    k = _key(args[0]) if args else None
    if op == "s_mov_b64" and k and args[1:2] == ["exec"]:
        ub2, orn2 = kill(dst)
        snap[k] = open_
        return St(open_, snap, ub2, orn2)
    if op == "s_xor_b64" and k and args[1:2] == ["exec"] and len(args) > 2 and args[2] == args[0] and k in st.snap:
        ub2, orn2 = kill(dst - {k})
        return St(open_, snap, ub2 - {k}, orn2 - {k})   # if-with-else: d = the else lanes, same restore
    if op == "s_cselect_b64" and k and set(args[1:3]) <= {"-1", "0"}:
        ub2, orn2 = kill(dst)
        return St(open_, snap, ub2 | {k}, orn2 | {k})
    if op == "s_mov_b64" and k and (args[1:2] in (["-1"], ["0"]) or _key(args[1]) in st.ub):
        ub2, orn2 = kill(dst)
        return St(open_, snap, ub2 | {k}, orn2 | {k})
    if op == "s_mov_b64" and k and _key(args[1]) in st.snap:
        ub2, orn2 = kill(dst)
        snap[k] = st.snap[_key(args[1])]
        return St(open_, snap, ub2, orn2)
    if op == "s_orn2_b64" and k and _key(args[1]) in st.ub and args[2:3] == ["exec"]:
        ub2, orn2 = kill(dst)
        return St(open_, snap, ub2, orn2 | {k})
    if op == "s_or_b64" and k and len(args) > 2 and args[0] in args[1:] and k in st.snap:
        # r |= more removed lanes (a loop's exit mask growing): EXEC | r still restores the saved state
        ub2, orn2 = kill(dst - {k})
        return St(open_, snap, ub2 - {k}, orn2 - {k})
    if dst:
        ub2, orn2 = kill(dst)
        return St(open_, snap, ub2, orn2)
    return st


def scan_function(body):
    """Indices of cross-lane instructions reached with an EXEC narrowing in force (forward dataflow over
    the function's CFG, module docstring)."""
    if not body:
        return []
    blocks = _blocks(body)
    ins = {0: St()}
    work = [0]
    while work:
        b = work.pop()
        st = ins[b]
        e, succ = blocks[b]
        for i in range(b, e + 1):
            st = _step(st, body[i][1], body[i][2], body[i][0])
        for s in succ:
            m = st if s not in ins else ins[s].merge(st)
            if s not in ins or not (ins[s] == m):
                ins[s] = m
                work.append(s)
    found = []
    for b, st in ins.items():
        e, _ = blocks[b]
        for i in range(b, e + 1):
            if CROSS_LANE.match(body[i][1]) and st.open:
                found.append(i)
            st = _step(st, body[i][1], body[i][2], body[i][0])
    return sorted(found)


def scan(lib: str, kernels=None):
    """[(function, address, instruction)] for every cross-lane op under a narrowed EXEC."""
    findings, counted = [], 0
    for text in disassemble(lib):
        for name, body in functions(text):
            if kernels and not any(k in name for k in kernels):
                continue
            counted += sum(1 for _, op, _ in body if CROSS_LANE.match(op))
            for i in scan_function(body):
                a, op, ops = body[i]
                findings.append((name, hex(a), f"{op} {ops}"))
    return findings, counted


def main(argv):
    lib = argv[1] if len(argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                     "channelestimationtransformer_amd", "libcet.so")
    findings, counted = scan(lib, argv[2:] or None)
    print(f"{counted} cross-lane permute/swap instructions scanned, {len(findings)} under a narrowed EXEC")
    for f in findings[:40]:
        print("  ", *f)
    return 1 if findings else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
