# round-6 session 8: the timing / placement race test (five production cases) on the committed build
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s8; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_race.py -v --timeout 120 --timeout-method thread > $O/race.log 2>&1
echo "race rc $?"; grep -E "PASSED|FAILED|passed|failed" $O/race.log | tail -7
