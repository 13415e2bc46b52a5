#!/bin/bash
# GPU tests, then the precision sweep over the fixtures, then the bench (each step time-limited).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v ${PYTEST_ARGS} --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/precision_check.py > gpurun_out/precision.jsonl 2> gpurun_out/precision.err
rc=$?; echo "precision rc=$rc"; cat gpurun_out/precision.jsonl; tail -3 gpurun_out/precision.err
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
echo "bench rc=$?"; tail -1 gpurun_out/bench.log
for v in 3 4; do timeout -k 10 300 python bench.py --steps 200 --warmup 100 --variant $v --no-cpu-baseline > gpurun_out/bench_v$v.log 2>&1 || exit 1; echo "v$v: $(python -c "import json;d=json.loads(open('gpurun_out/bench_v$v.log').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['kernel_ms'])")"; done
