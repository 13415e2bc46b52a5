#!/bin/bash
# layer-wise engine: GPU parity tests, the d64 config line, rocprofv3 kernel stats -> gpurun_out/$TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03_lw}; O=gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_layerwise.py tests/test_gpu_data.py -m gpu -q --maxfail=3 --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 "$O/gpu_tests.log")"
grep -E "^(FAILED|ERROR)" "$O/gpu_tests.log" | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python tools/bench_configs.py --only d64 --steps 50 > "$O/d64.jsonl" 2> "$O/prof.err" || { tail -5 "$O/prof.err"; exit 1; }
cut -c1-400 "$O/d64.jsonl"
find "$O/prof" -name "*kernel_stats.csv" -exec head -7 {} \; | cut -c1-140
