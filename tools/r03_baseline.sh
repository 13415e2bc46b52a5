#!/bin/bash
# Round-3 start: GPU suite, default bench line, and a rocprofv3 kernel trace of a short bench run
# (inter-dispatch gaps between back-to-back steps).   -> gpurun_out/r03_base/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_base; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 "$O/gpu_tests.log")"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err" || exit 1
cut -c1-400 "$O/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run -- python bench.py --steps 20 --warmup 5 --settle-s 0 --no-cpu-baseline > "$O/bench_trace.json" 2> "$O/trace.err" || exit 1
find "$O/trace" -name "*.csv" | head -20
