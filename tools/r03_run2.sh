#!/bin/bash
# probe v3 (data layout x scale rule), fp8 + informer GPU tests, bench inflight 2 vs 1 -> gpurun_out/r03_run2/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_run2; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 60 ./tools/probe/mfma_scale_probe > "$O/mfma_scale_probe.txt" 2>&1 || { echo "probe rc=$?"; cat "$O/mfma_scale_probe.txt"; exit 1; }
grep -v "raised" "$O/mfma_scale_probe.txt"
timeout -k 10 400 python -u -m pytest tests/test_gpu_informer.py -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 "$O/gpu_tests.log")"
grep -E "^(FAILED|ERROR)" "$O/gpu_tests.log" | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for n in 2 1; do
  timeout -k 10 300 python bench.py --inflight $n --no-cpu-baseline > "$O/bench_if$n.json" 2> "$O/bench_if$n.err" || { tail -5 "$O/bench_if$n.err"; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_if$n.json')); r=d['roofline']; print('inflight $n', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('achieved_from_throughput'), d['parity_rel_nmse_vs_oracle'], d['nmse_gathered_vs_allreduced_rel'])"
done
