set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=channelestimationtransformer_amd
O=gpurun_out/ab16; mkdir -p $O
for v in lnf; do
  CET_LIB=$(pwd)/$L/libcet_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_informer.py tests/test_gpu_inflight.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/tests_$v.log)"
done
bash tools/ab_bench.sh $L/libcet.so $L/libcet_lnf.so | tee $O/ab.log || exit 1
echo done
