set -o pipefail
cd "$GRAFT_REPO_ROOT"
L=channelestimationtransformer_amd
O=gpurun_out/ab5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_main.log 2>&1 || { tail -30 $O/tests_main.log; exit 1; }
echo "main $(tail -1 $O/tests_main.log)"
timeout -k 10 300 python -u tools/steps_probe.py 20 300 | tee $O/steps_probe.log || exit 1
bash tools/ab_bench.sh $L/libcet.so $L/libcet_new8.so | tee $O/ab.log || exit 1
bash tools/session.sh ab5 configs > /dev/null || exit 1; cat gpurun_out/ab5/configs.jsonl | cut -c1-400
echo done
