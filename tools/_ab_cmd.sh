set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=channelestimationtransformer_amd
O=gpurun_out/ab17; mkdir -p $O
CET_LIB=$(pwd)/$L/libcet_c2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_c2.log 2>&1 || { tail -30 $O/tests_c2.log; exit 1; }
echo "c2 $(tail -1 $O/tests_c2.log)"
bash tools/ab_bench.sh $L/libcet_base6.so $L/libcet_c2.so | tee $O/ab.log || exit 1
echo done
