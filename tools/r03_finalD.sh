#!/bin/bash
# Round-3 evidence after the fused layer-wise form: full GPU suite, smoke, default bench, every config line,
# rocprofv3 kernel stats of the d64 checkpoint-architecture forward   ->  gpurun_out/TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03_finalD}; O=gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 "$O/gpu_tests.log")"
[ $rc -eq 0 ] || { grep -E "FAILED|ERROR" "$O/gpu_tests.log" | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 || { tail -3 "$O/smoke.txt"; exit 1; }
tail -1 "$O/smoke.txt"
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -3 "$O/bench.err"; exit 1; }
echo "bench: $(tail -1 "$O/bench.json" | cut -c1-200)"
timeout -k 10 400 python tools/bench_configs.py > "$O/configs.jsonl" 2> "$O/configs.err" || { tail -3 "$O/configs.err"; exit 1; }
cut -c1-160 "$O/configs.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/d64prof" -o run -- python tools/bench_configs.py --only d64 --steps 50 > "$O/d64_under_rocprof.jsonl" 2> "$O/d64prof.err" || { tail -5 "$O/d64prof.err"; exit 1; }
find "$O/d64prof" -name "*kernel_stats.csv" -exec head -4 {} \; | cut -c1-200
