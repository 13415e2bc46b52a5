# round-6 session 13: the ab8 request order with the K/V tiles handed over in registers (-DCET_AB8 -DCET_AB8_EXTKV,
# correct: DESIGN §3.0e) as a performance candidate: same-box A/B against the default build, then its GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s13; mkdir -p $O
L=channelestimationtransformer_amd
AB_ROUNDS=3 timeout -k 10 600 bash tools/ab_bench.sh $L/libcet.so $L/libcet_ab8x.so 2>&1 | tee $O/ab_ab8x.log
CET_LIB=$(pwd)/$L/libcet_ab8x.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_ab8x.log 2>&1
echo "tests rc $?"; tail -2 $O/tests_ab8x.log
