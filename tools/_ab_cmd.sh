set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=channelestimationtransformer_amd
O=gpurun_out/ab18; mkdir -p $O
CET_LIB=$(pwd)/$L/libcet_c3.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_c3.log 2>&1 || { tail -30 $O/tests_c3.log; exit 1; }
echo "c3 $(tail -1 $O/tests_c3.log)"
for v in base7 c3; do CET_LIB=$(pwd)/$L/libcet_$v.so timeout -k 10 600 python tools/bench_configs.py > $O/configs_$v.jsonl 2> $O/configs_$v.err || { tail -5 $O/configs_$v.err; exit 1; }; echo "== $v"; python - $O/configs_$v.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d['config'][:40], d['kernel_ms'], d['seq_per_s'], d.get('parity_rel_nmse_vs_oracle'))
PY
done
echo done
