set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=channelestimationtransformer_amd
O=gpurun_out/lw4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_layerwise.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_lw8.log 2>&1 || { tail -30 $O/tests_lw8.log; exit 1; }
echo "lw8 $(tail -1 $O/tests_lw8.log)"
for i in 1 2; do for v in "" _lw8; do echo "libcet$v: $(CET_LIB=$(pwd)/$L/libcet$v.so timeout -k 10 120 python tools/d64_time.py 512 200)"; done; done | tee $O/d64.log
CET_LIB=$(pwd)/$L/libcet_lw8s.so timeout -k 10 120 python tools/lwf_stamps.py 512 > $O/lwf_stamps_lw8.txt 2>&1 || { tail -5 $O/lwf_stamps_lw8.txt; exit 1; }
tail -3 $O/lwf_stamps_lw8.txt
echo done
