# round-6 session 15: the default build with the early K/V request: the GPU suite, smoke(), the
# driver's bench command, the default bench and the rocprofv3 kernel statistics with one batch in flight
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s15; mkdir -p $O
bash tools/session.sh r06s15 tests smoke bench2 bench1 prof &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_args.json 2> $O/bench_driver_args.err &&
cut -c1-300 $O/bench_driver_args.json
