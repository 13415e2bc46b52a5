# round-6 session 2: the default library's GPU suite (poison, lab20 mixed and feed tests included), the ab8
# candidate plain and under the LDS poison, the lab20 mixed measurement, and the LN_LAST A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s2; mkdir -p $O
L=channelestimationtransformer_amd
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; echo "default suite rc $?"; tail -3 $O/gpu_tests.log; grep FAILED $O/gpu_tests.log | head
timeout -k 10 300 python tools/lab20_mixed.py 512 > $O/lab20_mixed.json 2> $O/lab20_mixed.err; echo "lab20 mixed rc $?"; cat $O/lab20_mixed.json
timeout -k 10 400 python tools/bench_configs.py --only lab20 > $O/configs_lab20.jsonl 2> $O/configs_lab20.err; echo "configs rc $?"; cut -c1-400 $O/configs_lab20.jsonl
K="split_bf16_is_fp32_parity or reference_fixture"
CET_LIB=$(pwd)/$L/libcet_ab8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_informer.py -k "$K" -v --timeout 120 --timeout-method thread > $O/ab8_plain.log 2>&1; echo "ab8 plain rc $?"; grep -E "passed|failed" $O/ab8_plain.log | tail -2
CET_LDS_POISON=1 CET_LIB=$(pwd)/$L/libcet_ab8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_informer.py -k "$K" -v --timeout 120 --timeout-method thread > $O/ab8_poison.log 2>&1; echo "ab8 poison rc $?"; grep -E "passed|failed" $O/ab8_poison.log | tail -2
CET_LIB=$(pwd)/$L/libcet_lnlast.so timeout -k 10 300 python -u -m pytest tests/test_gpu_informer.py tests/test_gpu_poison.py -x -q --timeout 120 --timeout-method thread > $O/lnlast_tests.log 2>&1; echo "lnlast tests rc $?"; tail -2 $O/lnlast_tests.log
AB_ROUNDS=3 bash tools/ab_bench.sh $L/libcet.so $L/libcet_lnlast.so 2>&1 | tee $O/ab_lnlast.log
bash tools/ab_configs.sh "e_layers=[4,3]" $L/libcet.so $L/libcet_lnlast.so 2>&1 | tee $O/ab_lnlast_e43.log
bash tools/stamps_ab.sh $O/stamps $L/libcet_c2st.so $L/libcet_c2st_lnlast.so
