#!/bin/bash
# One GPU call of kernel A/B work: parity of every candidate build (the fused-Informer GPU tests), the
# same-box alternated bench A/B, then the instruction-count PMC pass per build.
#   tools/ab_round.sh TAG lib_a.so lib_b.so ...      (paths relative to the repo root)
# Outputs under gpurun_out/TAG/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp
for L in "$@"; do
  n=$(basename "$L" .so)
  CET_LIB=$(pwd)/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_informer.py -x -q --timeout 120 \
    --timeout-method thread > "$O/tests_$n.log" 2>&1 || { echo "TESTS FAILED $n"; tail -30 "$O/tests_$n.log"; exit 1; }
  echo "$n: $(tail -1 "$O/tests_$n.log")"
done


bash tools/ab_bench.sh "$@" | tee "$O/ab.log" || exit 1
R=$(pwd)
for L in "$@"; do
  n=$(basename "$L" .so)
  (cd /tmp && CET_LIB=$R/$L timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS \
    SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT --output-format csv -d "$R/$O/pmc_$n" -o pmc -- \
    python "$R/tools/run_forward.py" 10 512 4 > /dev/null 2> "$R/$O/pmc_$n.err") || exit 1
  echo "== $n"; python tools/pmc_summary.py "$O/pmc_$n" informer_forward_v4
done
