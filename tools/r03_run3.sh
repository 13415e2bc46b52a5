#!/bin/bash
# full GPU suite, the other configs (C3, C5 bf16/fp8, full e43, d64), bench inflight 3, rocprofv3 stats of the
# default bench  -> gpurun_out/r03_run3/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_run3; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 "$O/gpu_tests.log")"
grep -E "^(FAILED|ERROR)" "$O/gpu_tests.log" | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python tools/bench_configs.py > "$O/configs.jsonl" 2> "$O/configs.err" || { echo "configs rc=$?"; tail -5 "$O/configs.err"; exit 1; }
python -c "
import json
for l in open('$O/configs.jsonl'):
    d=json.loads(l); print(d['config'][:60], d['batch'], d['precision'], d['seq_per_s'], d['kernel_ms'], d['mfma_frac'], d['parity_rel_nmse_vs_oracle'])"
timeout -k 10 300 python bench.py --inflight 3 --no-cpu-baseline > "$O/bench_if3.json" 2> "$O/bench_if3.err" || exit 1
python -c "import json; d=json.load(open('$O/bench_if3.json')); print('inflight 3', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python bench.py --steps 400 --warmup 100 --no-cpu-baseline > "$O/bench_prof.json" 2> "$O/prof.err" || exit 1
find "$O/prof" -name "*kernel_stats.csv" -exec head -3 {} \;
