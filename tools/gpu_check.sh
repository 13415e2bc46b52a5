# GPU box: parity tests, bench (default kernel + v2 for comparison) and per-phase stamps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cat gpurun_out/bench.json
timeout -k 10 200 python tools/ablate.py 3 2 > gpurun_out/ablate.txt 2>&1 || exit 1
cat gpurun_out/ablate.txt
timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps.txt 2>&1 || exit 1
cat gpurun_out/stamps.txt
