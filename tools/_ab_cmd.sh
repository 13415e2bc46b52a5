set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=channelestimationtransformer_amd
O=gpurun_out/lw1; mkdir -p $O
for v in lwA lwB lwC; do
  CET_LIB=$(pwd)/$L/libcet_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_layerwise.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/tests_$v.log)"
done
for i in 1 2; do for v in "" _lwA _lwB _lwC; do echo "libcet$v: $(CET_LIB=$(pwd)/$L/libcet$v.so timeout -k 10 120 python tools/d64_time.py 512 200)"; done; done | tee $O/d64.log
echo done
