#!/bin/bash
# Round-3 evidence, part C: the SNR sweep (C4 per rank, 200 reference batches per SNR) and the batch-1
# TimingAnalysis latency series + sweep (layer-wise shapes included)   -> gpurun_out/TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03_final}; O=gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python -m channelestimationtransformer_amd.sweep --batches 200 > "$O/sweep_200batches.jsonl" 2> "$O/sweep.err" || { tail -3 "$O/sweep.err"; exit 1; }
cut -c1-200 "$O/sweep_200batches.jsonl"
timeout -k 10 400 python -m channelestimationtransformer_amd.latency --series --reps 1000 > "$O/latency_series.jsonl" 2> "$O/latency_series.err" || { tail -3 "$O/latency_series.err"; exit 1; }
head -3 "$O/latency_series.jsonl" | cut -c1-200
timeout -k 10 700 python -m channelestimationtransformer_amd.latency --sweep --reps 300 > "$O/latency_sweep.jsonl" 2> "$O/latency_sweep.err" || { tail -3 "$O/latency_sweep.err"; exit 1; }
wc -l "$O/latency_sweep.jsonl"
