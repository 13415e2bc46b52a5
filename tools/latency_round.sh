#!/bin/bash
# Batch-1 latency evidence: the whole cumulative TimingAnalysis sweep, then a kernel trace of the timing
# config so the model-call time splits into kernel and dispatch.   bash tools/latency_round.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-lat}; O=gpurun_out/$TAG; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 600 python -m channelestimationtransformer_amd.latency --sweep --reps 300 > "$O/latency_sweep.jsonl" 2> "$O/latency.err" || exit 1
head -3 "$O/latency_sweep.jsonl" | cut -c1-260
R=$(pwd)
(cd /tmp && export PYTHONPATH="$R" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o trace -- \
  python -m channelestimationtransformer_amd.latency --reps 300 > "$R/$O/timing_config.jsonl" 2> "$R/$O/prof.err") || exit 1
cat "$O/timing_config.jsonl" | cut -c1-260
head -4 "$O"/prof/trace_kernel_stats.csv | cut -c1-200
