# round-6 session 10: the rebuilt tree as the round-end driver runs it: the GPU suite, smoke(), its bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s10; mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gpu_rccl.py -v --timeout 200 --timeout-method thread > $O/rccl.log 2>&1; echo "rccl rc $?"; tail -3 $O/rccl.log
bash tools/session.sh r06s10 tests smoke &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_args.json 2> $O/bench_driver_args.err &&
cut -c1-300 $O/bench_driver_args.json
