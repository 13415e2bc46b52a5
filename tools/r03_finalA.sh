#!/bin/bash
# Round-3 evidence, part A: full GPU suite, smoke, default bench + rocprofv3 stats + HBM PMC passes
#   bash tools/r03_finalA.sh TAG  -> gpurun_out/TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03_final}; O=gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 "$O/gpu_tests.log")"
[ $rc -eq 0 ] || { grep -E "FAILED|ERROR" "$O/gpu_tests.log" | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 || { tail -3 "$O/smoke.txt"; exit 1; }
tail -1 "$O/smoke.txt"
KERNEL=informer_forward_v4 bash tools/profile_round.sh "$TAG" || exit 1
echo "bench: $(tail -1 "$O/bench.json" | cut -c1-300)"
find "$O/prof" -name "*kernel_stats.csv" -exec head -3 {} \; | cut -c1-200
cat "$O/pmc_traffic.json" | head -20
