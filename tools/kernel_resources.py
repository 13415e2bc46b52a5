"""Register / scratch metadata of every kernel in the gfx950 code objects bundled in libcet.so (the
compiler's own record: .vgpr_count, .vgpr_spill_count, .sgpr_spill_count, .private_segment_fixed_size,
.group_segment_fixed_size), read from the code objects' AMDGPU metadata notes with llvm-readelf.

    python tools/kernel_resources.py [libcet.so] [name-substring ...]
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
FIELDS = ("vgpr_count", "vgpr_spill_count", "sgpr_count", "sgpr_spill_count", "private_segment_fixed_size",
          "group_segment_fixed_size")


def resources(lib: str) -> dict:
    """{mangled kernel name: {field: int}} over every gfx950 code object of `lib`."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        so = os.path.join(d, "lib.so")
        shutil.copy(lib, so)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", so], cwd=d, check=True, capture_output=True)
        for f in sorted(os.listdir(d)):
            if "amdgcn" not in f or "gfx950" not in f or os.path.getsize(os.path.join(d, f)) == 0:
                continue
            text = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", os.path.join(d, f)], check=True,
                                  capture_output=True, text=True).stdout
            # one kernel record per "- .agpr_count" list item of amdhsa.kernels
            for rec in re.split(r"\n\s*- \.agpr_count:", text)[1:]:
                name = re.search(r"\n\s*\.name:\s+(\S+)", rec)
                if not name:
                    continue
                vals = {}
                for k in FIELDS:
                    m = re.search(r"\n\s*\." + k + r":\s+(\d+)", rec)
                    if m:
                        vals[k] = int(m.group(1))
                out[name.group(1)] = vals
    return out


def main(argv):
    lib = argv[1] if len(argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                       "channelestimationtransformer_amd", "libcet.so")
    subs = argv[2:]
    for name, v in sorted(resources(lib).items()):
        if subs and not any(s in name for s in subs):
            continue
        print(" ".join(f"{k}={v.get(k, '-')}" for k in FIELDS), name)


if __name__ == "__main__":
    main(sys.argv)
