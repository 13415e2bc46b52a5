#!/bin/bash
# rocprofv3 kernel stats of the d64 (MimoSimulation checkpoint architecture) layer-wise forward at B=512
#   -> gpurun_out/r03_d64prof/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_d64prof; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python tools/bench_configs.py --only d64 --steps 50 > "$O/d64.jsonl" 2> "$O/prof.err" || { tail -5 "$O/prof.err"; exit 1; }
cat "$O/d64.jsonl"
find "$O/prof" -name "*kernel_stats.csv" -exec head -20 {} \;
