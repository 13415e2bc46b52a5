set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=channelestimationtransformer_amd
O=gpurun_out/ab7; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests $(tail -1 $O/tests.log)"
bash tools/ab_bench.sh $L/libcet_base5.so $L/libcet.so | tee $O/ab.log || exit 1
bash tools/session.sh ab7 traffic pmcinst stamps > /dev/null || exit 1
cat gpurun_out/ab7/pmc_traffic.json gpurun_out/ab7/pmcinst.txt; head -8 gpurun_out/ab7/stamps_b512.txt
echo done
