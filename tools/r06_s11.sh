# round-6 session 11: schedule-driven priority for the two workgroups of a CU (a throw-away build of
# -DCET_SCHED_PRIO=T, T = target ticks of the 100 MHz clock per workgroup) against the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s11; mkdir -p $O
L=channelestimationtransformer_amd
AB_ROUNDS=3 timeout -k 10 700 bash tools/ab_bench.sh $L/libcet.so $L/libcet_sp9500.so $L/libcet_sp10500.so 2>&1 | tee $O/ab_sched.log
