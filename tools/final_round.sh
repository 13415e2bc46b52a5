#!/bin/bash
# Round-end evidence on one GPU box: full GPU test suite, default bench + rocprofv3 stats + HBM PMC passes
# (tools/profile_round.sh), the other BASELINE configs, and the per-phase stamps of the DIAG instance.
#   bash tools/final_round.sh TAG     -> gpurun_out/TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-final}; O=gpurun_out/$TAG; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 "$O/gpu_tests.log")"
[ $rc -eq 0 ] || exit $rc
KERNEL=informer_forward_v4 bash tools/profile_round.sh "$TAG" || exit 1
echo "bench: $(tail -1 "$O/bench.json" | cut -c1-200)"
timeout -k 10 400 python tools/bench_configs.py > "$O/configs.jsonl" 2> "$O/configs.err" || exit 1
cat "$O/configs.jsonl" | cut -c1-220
timeout -k 10 200 python tools/stamps.py 512 > "$O/stamps_b512.txt" 2> "$O/stamps.err" || exit 1
head -3 "$O/stamps_b512.txt"
timeout -k 10 300 python -m channelestimationtransformer_amd.sweep --batches 200 > "$O/sweep_200batches.jsonl" 2> "$O/sweep.err" || exit 1
cut -c1-200 "$O/sweep_200batches.jsonl"
timeout -k 10 600 python -m channelestimationtransformer_amd.latency --sweep --reps 300 > "$O/latency_sweep.jsonl" 2> "$O/latency.err" || exit 1
head -2 "$O/latency_sweep.jsonl" | cut -c1-200
