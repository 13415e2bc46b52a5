#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v ${PYTEST_ARGS} --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/gpu_tests.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
  echo "bench rc=$?"
  tail -3 gpurun_out/bench.log
fi
