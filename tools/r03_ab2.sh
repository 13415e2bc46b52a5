#!/bin/bash
# A/B of the single-barrier decoder LayerNorm (libcet.so) against HEAD (libcet_base.so): the fused-Informer and
# Transformer GPU tests on the new build, the default bench line at one and two in flight alternated twice,
# then the d64 layer-wise profile   -> gpurun_out/r03_ab2/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_ab2; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_informer.py tests/test_gpu_transformer.py tests/test_gpu_layerwise.py -m gpu -q --maxfail=3 --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 "$O/gpu_tests.log")"
grep -E "^(FAILED|ERROR)" "$O/gpu_tests.log" | head -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for rep in 1 2; do
  for lib in base new; do
    L=channelestimationtransformer_amd/libcet.so; [ $lib = base ] && L=channelestimationtransformer_amd/libcet_base.so
    for n in 1 2; do
      CET_LIB=$PWD/$L timeout -k 10 200 python bench.py --inflight $n --steps 400 --no-cpu-baseline > "$O/b_${lib}_${n}_$rep.json" 2> "$O/b_${lib}_${n}_$rep.err" || { tail -3 "$O/b_${lib}_${n}_$rep.err"; exit 1; }
      python -c "import json; d=json.load(open('$O/b_${lib}_${n}_$rep.json')); r=d['roofline']; print('$lib inflight $n rep $rep', d['value'], d['ms_per_step'], r['kernel_ms'], d['parity_rel_nmse_vs_oracle'])"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/d64prof" -o run -- python tools/bench_configs.py --only d64 --steps 50 > "$O/d64.jsonl" 2> "$O/d64prof.err" || { tail -5 "$O/d64prof.err"; exit 1; }
cut -c1-300 "$O/d64.jsonl"
find "$O/d64prof" -name "*kernel_stats.csv" -exec head -8 {} \; | cut -c1-140
