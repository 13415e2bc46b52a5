# round-6 session 12: the device sampler's prepared tables with batches past one wave of workgroups
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s12; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_informer.py -k "prepared_tables_with_batches or samplers_share or native" -v --timeout 120 --timeout-method thread > $O/sampler.log 2>&1
echo "rc $?"; grep -E "PASSED|FAILED|passed|failed" $O/sampler.log | tail -8
