"""Build the in-tree HIP engine library for gfx950:  python -m channelestimationtransformer_amd.build"""
import os
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")


def build(jobs: int = 8) -> str:
    jobs = max(1, min(jobs, 16))
    subprocess.run(["make", "-C", CSRC, f"-j{jobs}"], check=True)
    lib = os.path.join(os.path.dirname(CSRC), "libcet.so")
    if not os.path.exists(lib):
        raise RuntimeError("libcet.so was not produced")
    return lib


if __name__ == "__main__":
    print(build(int(sys.argv[1]) if len(sys.argv) > 1 else 8))
