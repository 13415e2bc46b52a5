#!/bin/bash
# Round-3 iteration on one GPU box: the fused-Informer GPU tests (stop at the first failure), the default
# bench line for both kernel generations, and a rocprofv3 kernel-trace summary of the v5 bench.
#   bash tools/r03_iter.sh TAG [pytest-args...]   -> gpurun_out/TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-iter}; shift
O=gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp
T=${@:-tests -m gpu}
timeout -k 10 600 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 "$O/gpu_tests.log")"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" "$O/gpu_tests.log" | head -20; exit $rc; fi
for v in 5 4; do
  timeout -k 10 300 python bench.py --variant $v --no-cpu-baseline > "$O/bench_v$v.json" 2> "$O/bench_v$v.err" || exit 1
  python -c "import json,sys; d=json.load(open('$O/bench_v$v.json')); r=d['roofline']; print('v$v', d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms'], r['frac'], d['parity_rel_nmse_vs_oracle'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$O/bench_prof.json" 2> "$O/prof.err" || exit 1
find "$O/prof" -name "*kernel_stats.csv" -exec head -4 {} \;
