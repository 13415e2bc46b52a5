set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=channelestimationtransformer_amd
O=gpurun_out/ab3; mkdir -p $O
CET_LIB=$(pwd)/$L/libcet_new4.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_new4.log 2>&1 || { tail -30 $O/tests_new4.log; exit 1; }
tail -1 $O/tests_new4.log
bash tools/ab_bench.sh $L/libcet_new2.so $L/libcet_new3.so $L/libcet_new4.so | tee $O/ab.log || exit 1
for v in new3 new4; do CET_LIB=$(pwd)/$L/libcet_$v.so bash tools/session.sh ab3_$v pmcvalu > /dev/null || exit 1; done
CET_LIB=$(pwd)/$L/libcet_new4.so bash tools/session.sh ab3_new4 stamps traffic > /dev/null || exit 1
cat gpurun_out/ab3_new3/pmcvalu.txt gpurun_out/ab3_new4/pmcvalu.txt
echo done
