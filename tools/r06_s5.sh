# round-6 session 5: (1) the ab8 candidate with and without 32 wait states between the attention's K/V MFMA
# chains and their VALU epilogue (-DCET_MFMA_NOP); (2) the straight-line sparsity measurement (libcet_mq.so):
# its tests, then a same-box A/B against the committed build
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s5; mkdir -p $O
L=channelestimationtransformer_amd
for v in ab8 ab8nop; do
  CET_LIB=$(pwd)/$L/libcet_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_informer.py -k "split_bf16_is_fp32_parity" -v --timeout 120 --timeout-method thread > $O/$v.log 2>&1; echo "$v rc $?"; grep -E "passed|failed" $O/$v.log | tail -1
done
CET_LIB=$(pwd)/$L/libcet_mq.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/mq_tests.log 2>&1
echo "mq tests rc $?"; tail -2 $O/mq_tests.log
timeout -k 10 600 bash tools/ab_bench.sh $L/libcet.so $L/libcet_mq.so 2>&1 | tee $O/ab_mq.log
timeout -k 10 600 bash tools/stamps_ab.sh $O/stamps $L/libcet_c2st.so $L/libcet_c2st_mq.so
