# round-6 session 9: the private-memory reload probe (tools/probe/scratch_probe.hip), and the ab8 build with the
# vector L1 invalidated before its K/V struct is read back from private memory (-DCET_AB8_INV)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s9; mkdir -p $O
timeout -k 10 300 hipcc --offload-arch=gfx950 -O3 -Wno-unused-result tools/probe/scratch_probe.hip -o $O/scratch_probe || exit 1
timeout -k 10 120 $O/scratch_probe 64 4 20 > $O/probe_short.txt 2>&1; echo "short rc $?"; tail -3 $O/probe_short.txt
timeout -k 10 180 $O/scratch_probe 256 8 100 > $O/probe_long.txt 2>&1; echo "long rc $?"; tail -3 $O/probe_long.txt
L=channelestimationtransformer_amd
for v in ab8 ab8inv; do
  CET_LIB=$(pwd)/$L/libcet_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_informer.py -k "split_bf16_is_fp32_parity" -v --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1
  echo "parity $v rc $?"; grep -E "passed|failed" $O/parity_$v.log | tail -1
done
