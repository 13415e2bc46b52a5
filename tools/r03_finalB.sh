#!/bin/bash
# Round-3 evidence, part B: the kernel alone (one batch in flight) + its rocprofv3 stats, the other
# BASELINE configs, the DIAG per-phase stamps   -> gpurun_out/TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03_final}; O=gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --inflight 1 > "$O/bench_inflight1.json" 2> "$O/bench_inflight1.err" || exit 1
cut -c1-200 "$O/bench_inflight1.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_if1" -o trace -- python bench.py --inflight 1 --steps 200 --warmup 100 --no-cpu-baseline > "$O/prof_if1_bench.json" 2> "$O/prof_if1.err" || exit 1
find "$O/prof_if1" -name "*kernel_stats.csv" -exec head -3 {} \; | cut -c1-200
timeout -k 10 500 python tools/bench_configs.py > "$O/configs.jsonl" 2> "$O/configs.err" || { tail -3 "$O/configs.err"; exit 1; }
cut -c1-250 "$O/configs.jsonl"
timeout -k 10 200 python tools/stamps.py 512 > "$O/stamps_b512.txt" 2> "$O/stamps.err" || exit 1
head -3 "$O/stamps_b512.txt"
