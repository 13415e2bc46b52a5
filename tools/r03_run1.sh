#!/bin/bash
# Round-3 GPU call: scaled-MFMA layout probe, GPU suite, default bench line, and a rocprofv3 kernel
# trace of a short bench run (inter-dispatch gaps between back-to-back steps).  -> gpurun_out/$TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03_run1}
O=gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 60 ./tools/probe/mfma_scale_probe > "$O/mfma_scale_probe.txt" 2>&1 || { echo "probe rc=$?"; cat "$O/mfma_scale_probe.txt"; exit 1; }
cat "$O/mfma_scale_probe.txt"
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 "$O/gpu_tests.log")"
grep -E "^(FAILED|ERROR)" "$O/gpu_tests.log" | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err" || exit 1
cut -c1-300 "$O/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run -- python bench.py --steps 20 --warmup 5 --settle-s 0 --no-cpu-baseline > "$O/bench_trace.json" 2> "$O/trace.err" || exit 1
find "$O/trace" -name "*.csv" | head -20
