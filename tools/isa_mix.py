"""Static instruction mix of kernels in a gfx950 assembly file (hipcc --save-temps):
python tools/isa_mix.py file.s [substring-of-kernel-name ...]"""
import sys


def kernels(path):
    cur, out = None, {}
    for line in open(path):
        s = line.split(";")[0].strip()
        if s.endswith(":") and not s.startswith(".") and s[:-1].startswith("_Z"):
            cur = s[:-1]
            out[cur] = {}
            continue
        if cur is None:
            continue
        if s.startswith("s_endpgm"):
            cur = None
            continue
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        k = ("mfma" if "mfma" in op else "scratch" if op.startswith("scratch") else
             "ds" if op.startswith("ds_") else "vmem" if op.startswith(("buffer", "global")) else
             "smem" if op.startswith("s_load") or op.startswith("s_buffer") else
             "barrier" if op == "s_barrier" else "waitcnt" if op.startswith("s_waitcnt") else
             "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "other")
        out[cur][k] = out[cur].get(k, 0) + 1
    return out


if __name__ == "__main__":
    ks = kernels(sys.argv[1])
    for name, c in ks.items():
        if len(sys.argv) > 2 and not any(p in name for p in sys.argv[2:]):
            continue
        print(name[:70], dict(sorted(c.items())))
