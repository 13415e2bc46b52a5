#!/bin/bash
# Same-box A/B of libcet_base.so (HEAD) against the working-tree libcet.so: the fused-Informer GPU tests on
# the new build, then the default bench line at one and two batches in flight, alternated twice.
#   bash tools/r03_ab.sh TAG [test-selection]  -> gpurun_out/TAG/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-ab}; SEL=${2:-tests/test_gpu_informer.py}
O=gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest $SEL -m gpu -q --maxfail=3 --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
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
