# round-6 session 18: the Q weights added to the early K/V request (-DCET_EARLY_Q; C2 spills 12 -> 71 VGPRs) against
# the default build, alternated on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s18; mkdir -p $O
L=channelestimationtransformer_amd
AB_ROUNDS=2 timeout -k 10 600 bash tools/ab_bench.sh $L/libcet.so $L/libcet_eq.so 2>&1 | tee $O/ab_early_q.log
