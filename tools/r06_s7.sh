# round-6 session 7: (1) the timing / placement race test on the committed build; (2) the ab8 candidate with its
# K/V weight struct in private memory (libcet_ab8.so) and with the K/V tiles handed over in registers
# (libcet_ab8x.so: -DCET_AB8_EXTKV, no private memory): the split-bf16 parity test and the race test on each;
# (3) the committed tree end to end (tools/r06_s6.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s7; mkdir -p $O
L=channelestimationtransformer_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_race.py -v --timeout 120 --timeout-method thread > $O/race_base.log 2>&1
echo "race base rc $?"; grep -E "passed|failed" $O/race_base.log | tail -1
for v in ab8 ab8x; do
  CET_LIB=$(pwd)/$L/libcet_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_informer.py -k "split_bf16_is_fp32_parity" -v --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1
  echo "parity $v rc $?"; grep -E "passed|failed" $O/parity_$v.log | tail -1
  CET_LIB=$(pwd)/$L/libcet_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_race.py -k split -v --timeout 120 --timeout-method thread > $O/race_$v.log 2>&1
  echo "race $v rc $?"; grep -E "passed|failed" $O/race_$v.log | tail -1
done
bash tools/r06_s6.sh
