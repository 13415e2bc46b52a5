cd $GRAFT_REPO_ROOT
L=channelestimationtransformer_amd/libcet_stag.so
for i in 1 2; do
for sg in 0 $((256*65536+300)) $((256*65536+800)) $((256*65536+1600)) $((1*65536+800)) $((1*65536+1600)); do
  r=$(CET_STAGGER=$sg CET_LIB=$(pwd)/$L timeout -k 10 120 python bench.py --steps 300 --warmup 100 --no-cpu-baseline 2>/dev/null | tail -1) || exit 1
  echo "stagger $sg: $(echo "$r" | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
done; done
