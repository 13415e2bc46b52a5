set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=channelestimationtransformer_amd
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err || exit 1
cut -c1-200 $O/bench.json $O/bench_steps20.json
CET_LIB=$(pwd)/$L/libcet_lwg.so timeout -k 10 600 python -u -m pytest tests/test_gpu_layerwise.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_lwg.log 2>&1 || { tail -30 $O/tests_lwg.log; exit 1; }
echo "lwg $(tail -1 $O/tests_lwg.log)"
for i in 1 2; do for v in _lwbase _lwg; do echo "libcet$v: $(CET_LIB=$(pwd)/$L/libcet$v.so timeout -k 10 120 python tools/d64_time.py 512 200)"; done; done | tee $O/d64.log
echo done
