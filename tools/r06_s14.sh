# round-6 session 14: the early K/V request with register hand-over (libcet_ab8x.so) against the default build at
# the driver's bench command (--steps 20 --warmup 5), alternated four times on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s14; mkdir -p $O
L=channelestimationtransformer_amd
for i in 1 2 3 4; do
  for lib in libcet.so libcet_ab8x.so; do
    r=$(CET_LIB=$(pwd)/$L/$lib timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | tail -1) || exit 1
    echo "$lib: $(echo "$r" | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")" | tee -a $O/ab_steps20.log
  done
done
