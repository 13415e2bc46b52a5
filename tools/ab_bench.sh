#!/bin/bash
# Same-box A/B of bench.py kernel time: tools/ab_bench.sh "LIB:VARIANT" "LIB:VARIANT" ... (alternated twice);
# BENCH_ARGS adds bench.py options (e.g. "--nmse separate").
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for spec in "$@"; do
    lib=${spec%%:*}; var=${spec##*:}
    r=$(CET_LIB=$(pwd)/$lib timeout -k 10 120 python bench.py --steps 300 --warmup 100 --variant $var --no-cpu-baseline $BENCH_ARGS 2>/dev/null | tail -1) || exit 1
    echo "$lib v$var: $(echo "$r" | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['roofline']['kernel_ms'])")"
  done
done
