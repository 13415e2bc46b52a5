set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=channelestimationtransformer_amd
O=gpurun_out/ab9; mkdir -p $O
for v in ln6 ln3 embw; do
  CET_LIB=$(pwd)/$L/libcet_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_informer.py tests/test_gpu_inflight.py tests/test_gpu_transformer.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/tests_$v.log)"
done
bash tools/ab_bench.sh $L/libcet.so $L/libcet_ln6.so $L/libcet_ln3.so $L/libcet_embw.so | tee $O/ab.log || exit 1

CET_LIB=$(pwd)/$L/libcet_lwt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_layerwise.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_lwt.log 2>&1 || { tail -30 $O/tests_lwt.log; exit 1; }
echo "lwt $(tail -1 $O/tests_lwt.log)"
for i in 1 2; do for v in _lwbase _lwt; do echo "libcet$v: $(CET_LIB=$(pwd)/$L/libcet$v.so timeout -k 10 120 python tools/d64_time.py 512 200)"; done; done | tee $O/d64.log
echo done
