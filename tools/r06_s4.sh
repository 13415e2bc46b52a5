# round-6 session 4: the ab8 candidate with and without 32 wait states between the attention's K/V MFMA chains and
# their VALU epilogue (-DCET_MFMA_NOP): does the wrong V element go away?
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s4; mkdir -p $O
L=channelestimationtransformer_amd
for v in ab8 ab8nop; do
  CET_LIB=$(pwd)/$L/libcet_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_informer.py -k "split_bf16_is_fp32_parity" -v --timeout 120 --timeout-method thread > $O/$v.log 2>&1; echo "$v rc $?"; grep -E "passed|failed" $O/$v.log | tail -1
done
