set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/session.sh r04e tests smoke bench2 bench1 prof traffic pmcinst pmcwait stamps configs || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r04e/bench_steps20.json 2> gpurun_out/r04e/bench_steps20.err || exit 1
cut -c1-300 gpurun_out/r04e/bench_steps20.json
echo done
