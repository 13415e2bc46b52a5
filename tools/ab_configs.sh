#!/bin/bash
# Same-box A/B of tools/bench_configs.py lines: tools/ab_configs.sh ONLY LIB [LIB ...] (alternated AB_ROUNDS times)
cd "$GRAFT_REPO_ROOT"
ONLY=$1; shift
for i in $(seq 1 ${AB_ROUNDS:-2}); do
  for lib in "$@"; do
    r=$(CET_LIB=$(pwd)/$lib timeout -k 10 200 python tools/bench_configs.py --only "$ONLY" 2>/dev/null | tail -1) || exit 1
    echo "$lib: $(echo "$r" | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['seq_per_s'], d['kernel_ms'], d.get('parity_rel_nmse_vs_oracle'))")"
  done
done
