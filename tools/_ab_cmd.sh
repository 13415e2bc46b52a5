set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=channelestimationtransformer_amd
O=gpurun_out/ab2; mkdir -p $O
CET_LIB=$(pwd)/$L/libcet_new2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_new2.log 2>&1 || { tail -30 $O/tests_new2.log; exit 1; }
tail -1 $O/tests_new2.log
bash tools/ab_bench.sh $L/libcet_base.so $L/libcet_new.so $L/libcet_new2.so | tee $O/ab.log || exit 1
CET_LIB=$(pwd)/$L/libcet_new2.so bash tools/session.sh ab2_new2 pmcinst pmcwait pmcvalu stamps > /dev/null || exit 1
CET_LIB=$(pwd)/$L/libcet_base.so bash tools/session.sh ab2_base pmcvalu > /dev/null || exit 1
cat gpurun_out/ab2_new2/pmcvalu.txt gpurun_out/ab2_base/pmcvalu.txt
echo done
