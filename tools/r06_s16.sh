# round-6 session 16: the default build (early K/V request) against -DCET_LATE_KV (the previous order) at the
# driver's bench command, alternated six times on one box, then three times at 300 steps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s16; mkdir -p $O
L=channelestimationtransformer_amd
for i in 1 2 3 4 5 6; do
  for lib in libcet_late.so libcet.so; do
    r=$(CET_LIB=$(pwd)/$L/$lib timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | tail -1) || exit 1
    echo "$lib: $(echo "$r" | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")" | tee -a $O/ab_steps20.log
  done
done
AB_ROUNDS=3 timeout -k 10 600 bash tools/ab_bench.sh $L/libcet_late.so $L/libcet.so 2>&1 | tee $O/ab_steps300.log
