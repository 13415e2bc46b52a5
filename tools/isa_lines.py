"""Static instruction counts of one kernel per source line (innermost .loc), from a gfx950 assembly
file built with -gline-tables-only:  python tools/isa_lines.py i4g.s KERNEL_SUBSTR [N] [file-filter]"""
import collections
import re
import sys


def main():
    path, kname = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    files, loc, inside = {}, None, False
    cnt = collections.defaultdict(collections.Counter)
    for line in open(path):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', line)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
        if line.startswith("_Z") and kname in line.split(":")[0]:
            inside = True
            continue
        if not inside:
            continue
        s = line.split(";")[0].strip()
        if s.startswith("s_endpgm"):
            break
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            loc = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
            continue
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        k = ("mfma" if "mfma" in op else "ds" if op.startswith("ds_") else
             "vmem" if op.startswith(("buffer", "global", "scratch")) else
             "valu" if op.startswith("v_") else "salu")
        cnt[loc][k] += 1
    rows = sorted(cnt.items(), key=lambda kv: -kv[1]["valu"])
    tot = collections.Counter()
    for _, c in cnt.items():
        tot.update(c)
    print("total", dict(tot))
    for where, c in rows[:top]:
        print(f"{c['valu']:6d} valu {c['salu']:5d} salu {c['mfma']:4d} mfma {c['ds']:4d} ds {c['vmem']:4d} vmem  {where}")


if __name__ == "__main__":
    main()
