#!/bin/bash
# Bench + rocprofv3 kernel trace + HBM PMC passes for one round; outputs under gpurun_out/.
# usage (on the GPU box, from the repo root): bash tools/profile_round.sh r01
set -euo pipefail
TAG=${1:-r01}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 420 python "$R/bench.py" --steps 200 --warmup 100 > "$O/bench.json" 2> "$O/bench.err"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o trace -- \
  python "$R/bench.py" --steps 50 --warmup 5 --no-cpu-baseline > "$O/prof_bench.json" 2> "$O/prof.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o pmc -- \
  python "$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> "$O/pmc_fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o pmc -- \
  python "$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> "$O/pmc_write.err"

cd "$R" && python tools/pmc_traffic.py "$O" --kernel "${KERNEL:-informer_forward_v4}" --batch 512 -o "$O/pmc_traffic.json" > /dev/null
echo done > "$O/DONE"
