#!/bin/bash
# fp8 MFMA form A/B: the default build (v_mfma_f32_16x16x32_fp8_fp8 pairs) against -DCET_FP8_SCALED
# (libcet_fp8s.so, block-scaled 16x16x128): the fp8 GPU tests and the C5 lines of each  -> gpurun_out/r03_fp8ab/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_fp8ab; mkdir -p "$O"
export TMPDIR=/tmp
for lib in default fp8s; do
  L=$PWD/channelestimationtransformer_amd/libcet.so; [ $lib = fp8s ] && L=$PWD/channelestimationtransformer_amd/libcet_fp8s.so
  CET_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_informer.py -m gpu -q -k "fp8 or lsq" --timeout 120 --timeout-method thread > "$O/tests_$lib.log" 2>&1
  echo "$lib pytest rc=$?: $(tail -1 "$O/tests_$lib.log")"
  CET_LIB=$L timeout -k 10 400 python tools/bench_configs.py --only C5 > "$O/c5_$lib.jsonl" 2> "$O/c5_$lib.err" || { tail -3 "$O/c5_$lib.err"; exit 1; }
  python -c "
import json
for l in open('$O/c5_$lib.jsonl'):
    d=json.loads(l); print('$lib', d['config'][-22:], d['kernel_ms'], d['seq_per_s'], d['seq_per_s_two_in_flight'], d['mfma_frac'], '%.2e' % d['parity_rel_nmse_vs_oracle'])"
done
