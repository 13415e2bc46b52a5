# round-6 session 3: the TimingAnalysis e_layers [4,3] stack at B = 512 whole-sequence (default) against its
# encoder split (CET_SPLIT_MAX=1024: 1,024 workgroups, the last arrival runs the decoder), alternated
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s3; mkdir -p $O
for i in 1 2 3; do
  for sm in 512 1024; do
    CET_SPLIT_MAX=$sm timeout -k 10 200 python tools/bench_configs.py --only "FullPrecision InformerStack attn=full" > $O/cfg_${sm}_$i.jsonl 2> $O/cfg_${sm}_$i.err || { tail -20 $O/cfg_${sm}_$i.err; exit 1; }; r=$(head -1 $O/cfg_${sm}_$i.jsonl)
    echo "split_max $sm: $(echo "$r" | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['seq_per_s'], d['kernel_ms'], d.get('parity_rel_nmse_vs_oracle'), d.get('kernel'))")" | tee -a $O/ab_split.log
  done
done
CET_SPLIT_MAX=1024 timeout -k 10 300 python -u -m pytest tests/test_gpu_informer.py -k "encoder_split or e43" -q --timeout 120 --timeout-method thread > $O/split_tests.log 2>&1; echo "split tests rc $?"; tail -2 $O/split_tests.log
# final-tree evidence (C2 and the configs): smoke, the default bench (two in flight), the kernel alone, the
# driver's 20-step line, rocprofv3 kernel stats, PMC traffic / busy / instructions / waits, the batch-1 latency
# series and every config line
bash tools/session.sh r06final smoke bench2 bench1 prof traffic pmcbusy pmcinst pmcwait || exit 1
F=gpurun_out/r06final
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $F/bench_steps20.json 2> $F/bench20.err || exit 1; cut -c1-300 $F/bench_steps20.json
timeout -k 10 300 python -m channelestimationtransformer_amd.latency --series --reps 1000 > $F/latency_series.jsonl 2> $F/latency.err || exit 1; tail -3 $F/latency_series.jsonl
bash tools/session.sh r06final configs
