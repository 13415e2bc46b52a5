set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=channelestimationtransformer_amd
O=gpurun_out/lw10; mkdir -p $O
CET_LIB=$(pwd)/$L/libcet_fix.so CET_LW_FUSED_WHY=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_layerwise.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_fix.log 2>&1 || { tail -30 $O/tests_fix.log; exit 1; }
echo "fix $(tail -1 $O/tests_fix.log)"; grep -c "compile-time d64 layout yes" $O/tests_fix.log || true
for i in 1 2; do for v in _lwbase _fix; do echo "libcet$v: $(CET_LIB=$(pwd)/$L/libcet$v.so timeout -k 10 120 python tools/d64_time.py 512 200)"; done; done | tee $O/d64.log
echo done
