set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/v5l; mkdir -p $O
CET_NO_ENC_SPLIT=1 timeout -k 10 300 python tools/v5_debug.py > $O/debug.txt 2>&1 || { echo "debug rc=$?"; tail -5 $O/debug.txt; exit 1; }
grep -v Warn $O/debug.txt | grep -v amdgpu.ids | cut -c1-110
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $O/gpu_tests.log)"
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/gpu_tests.log | head -20; exit $rc; }
for v in 4 5; do
  timeout -k 10 300 python bench.py --variant $v --no-cpu-baseline > $O/bench_v$v.json 2> $O/bench_v$v.err || exit 1
  python -c "import json,sys; d=json.load(open('$O/bench_v$v.json')); r=d['roofline']; print('v$v', d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms'], r['frac'], d['parity_rel_nmse_vs_oracle'])"
done
