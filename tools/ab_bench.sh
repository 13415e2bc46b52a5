#!/bin/bash
# Same-box A/B of bench.py: tools/ab_bench.sh LIB [LIB ...] (alternated twice).  Per build: the default
# two-in-flight throughput and the kernel-alone time (roofline.kernel_ms); BENCH_ARGS adds bench.py options.
cd "$GRAFT_REPO_ROOT"
for i in $(seq 1 ${AB_ROUNDS:-2}); do
  for lib in "$@"; do
    r=$(CET_LIB=$(pwd)/$lib timeout -k 10 120 python bench.py --steps 300 --warmup 100 --no-cpu-baseline $BENCH_ARGS 2>/dev/null | tail -1) || exit 1
    echo "$lib: $(echo "$r" | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
  done
done
