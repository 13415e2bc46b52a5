set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/session.sh r04i tests smoke bench1 prof traffic pmcinst pmcwait stamps configs || exit 1
cp gpurun_out/r04i/pmc_traffic.json profiles/r04/pmc_traffic.json
timeout -k 10 300 python bench.py > gpurun_out/r04i/bench.json 2> gpurun_out/r04i/bench.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r04i/bench_steps20.json 2> gpurun_out/r04i/bench_steps20.err || exit 1
cut -c1-250 gpurun_out/r04i/bench.json gpurun_out/r04i/bench_steps20.json
echo done
