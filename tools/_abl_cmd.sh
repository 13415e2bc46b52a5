set -o pipefail
cd "$GRAFT_REPO_ROOT"
for l in abl_ln abl_mvalu abl_topu abl_gelu abl_dec ln1p; do
  CET_LIB=$(pwd)/channelestimationtransformer_amd/libcet_$l.so bash tools/session.sh abl_$l pmcinst pmcwait > /dev/null || exit 1
  echo "$l done"
done
CET_LIB=$(pwd)/channelestimationtransformer_amd/libcet_ln1p.so timeout -k 10 300 python -u -m pytest tests/test_gpu_informer.py tests/test_gpu_transformer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abl_ln1p/tests.log 2>&1; tail -2 gpurun_out/abl_ln1p/tests.log
bash tools/ab_bench.sh channelestimationtransformer_amd/libcet_base.so channelestimationtransformer_amd/libcet_ln1p.so | tee gpurun_out/ab_ln1p.log
