set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_informer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/q_tests.log; exit 1; }
tail -2 gpurun_out/q_tests.log
timeout -k 10 200 python tools/ablate.py 3 > gpurun_out/q_ablate.txt 2>&1 || { cat gpurun_out/q_ablate.txt; exit 1; }
cat gpurun_out/q_ablate.txt
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/q_bench_dev.json 2>gpurun_out/q_bench.err || exit 1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --sampler host > gpurun_out/q_bench_host.json 2>>gpurun_out/q_bench.err || exit 1
python -c "import json; [print(f, json.load(open('gpurun_out/'+f))['value'], json.load(open('gpurun_out/'+f))['roofline']['kernel_ms']) for f in ('q_bench_dev.json','q_bench_host.json')]"
