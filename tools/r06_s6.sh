# round-6 session 6: the committed tree end to end (the round-end driver's steps): the GPU suite, smoke(), the
# driver's bench command, the default bench, and the rocprofv3 kernel statistics of the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s6; mkdir -p $O
bash tools/session.sh r06s6 tests smoke bench2 prof2 &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_args.json 2> $O/bench_driver_args.err &&
cut -c1-300 $O/bench_driver_args.json
