#!/bin/bash
# Quick whole-tree check on one GPU box: the GPU test suite, smoke(), the default bench line and the
# batch-1 TimingAnalysis config.   bash tools/check_round.sh TAG  -> gpurun_out/TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-check}; O=gpurun_out/$TAG; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 "$O/gpu_tests.log")"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 || exit 1
cat "$O/smoke.txt" | tail -1
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err" || exit 1
tail -1 "$O/bench.json" | cut -c1-160
timeout -k 10 300 python -m channelestimationtransformer_amd.latency --series --reps 1000 > "$O/latency_series.jsonl" 2> "$O/latency.err" || exit 1
cut -c1-200 "$O/latency_series.jsonl"
