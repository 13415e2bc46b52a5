#!/bin/bash
# scale-reach probe of the block-scaled MFMA + the two-stream overlap experiment -> gpurun_out/r03_probe2/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_probe2; mkdir -p "$O"
timeout -k 10 60 ./tools/probe/mfma_scale_probe > "$O/mfma_scale_probe.txt" 2>&1 || { echo "probe rc=$?"; cat "$O/mfma_scale_probe.txt"; exit 1; }
cat "$O/mfma_scale_probe.txt"
timeout -k 10 300 python tools/overlap_probe.py 400 > "$O/overlap.jsonl" 2> "$O/overlap.err" || { echo "overlap rc=$?"; tail -5 "$O/overlap.err"; exit 1; }
cat "$O/overlap.jsonl"
