set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=channelestimationtransformer_amd
mkdir -p gpurun_out/ab1
CET_LIB=$(pwd)/$L/libcet_new.so timeout -k 10 400 python -u -m pytest tests/test_gpu_informer.py tests/test_gpu_transformer.py tests/test_gpu_inflight.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab1/tests_new.log 2>&1 || { tail -30 gpurun_out/ab1/tests_new.log; exit 1; }
tail -1 gpurun_out/ab1/tests_new.log
bash tools/ab_bench.sh $L/libcet_base.so $L/libcet_new.so $L/libcet_nocq.so $L/libcet_ln2b.so $L/libcet_earlyq.so | tee gpurun_out/ab1/ab.log || exit 1
for n in base new nocq ln2b earlyq; do
  CET_LIB=$(pwd)/$L/libcet_$n.so bash tools/session.sh ab1_$n pmcinst pmcwait > /dev/null || exit 1
done
echo done
