set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/session.sh r04h tests smoke configs || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r04h/bench.json 2> gpurun_out/r04h/bench.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r04h/bench_steps20.json 2> gpurun_out/r04h/bench_steps20.err || exit 1
cut -c1-250 gpurun_out/r04h/bench.json gpurun_out/r04h/bench_steps20.json
echo done
