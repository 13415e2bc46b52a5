"""Where a kernel's VGPR spills sit: scratch instructions of one kernel in a gfx950 assembly file
built with -gline-tables-only, grouped by the source line of the nearest .loc (inlined code keeps
the innermost file:line).

    hipcc ... --cuda-device-only -S -gline-tables-only cet_informer4_bf16.hip -o i4g.s
    python tools/spill_map.py i4g.s informer_forward_v4ILi64ELb0ELi0E
"""
import collections
import re
import sys


def main():
    path, kname = sys.argv[1], sys.argv[2]
    files, loc, inside = {}, None, False
    cnt = collections.Counter()
    for line in open(path):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', line)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
        if line.startswith("_Z") and kname in line.split(":")[0]:
            inside = True
            continue
        if not inside:
            continue
        s = line.strip()
        if s.startswith("s_endpgm"):
            break
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
        if m:
            loc = (files.get(m.group(1), m.group(1)), int(m.group(2)))
            continue
        if s.startswith("scratch_"):
            cnt[(loc, s.split()[0])] += 1
    for (where, op), n in sorted(cnt.items(), key=lambda kv: (kv[0][0] or ("", 0), kv[0][1])):
        print(f"{n:4d}  {op:22s} {where[0]}:{where[1]}" if where else f"{n:4d} {op}")
    print("total", sum(cnt.values()))


if __name__ == "__main__":
    main()
