#!/bin/bash
# One GPU call of a round's work, as named steps (run in order; the call stops at the first failure):
#   tools/session.sh TAG step [step ...]         outputs under gpurun_out/TAG/
# steps:
#   tests      full `pytest -m gpu` suite            bench1   bench.py --inflight 1 (kernel alone)
#   smoke      __graft_entry__ smoke()               bench2   bench.py (default: two batches in flight)
#   prof       rocprofv3 --kernel-trace --stats over bench.py --inflight 1
#   prof2      the same over the default bench.py
#   pmcwait    SQ wait / issue breakdown (one PMC pass)   pmcinst  instruction counts (one PMC pass)
#   pmcvalu    VALU instructions by kind (float add/mul/fma/transcendental, conversions, integer)
#   traffic    FETCH_SIZE and WRITE_SIZE passes -> traffic.json
#   stamps     DIAG per-phase stamps at B=512         configs  tools/bench_configs.py
#   stampsc2   C2-instance per-phase stamps at B=512 (libcet_c2st.so: make OUT=../libcet_c2st.so
#              B=build_c2st EXTRA=-DCET_C2_STAMPS)
#   list       rocprofv3 -L (counter names)
# CET_LIB in the environment selects an A/B build of the engine for every step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p "$O"
R=$(pwd)
export TMPDIR=/tmp
T="timeout -k 10"
fwd() { echo "python $R/tools/run_forward.py 10 512 4"; }
for s in "$@"; do
  echo "== $s $(date +%T)"
  case $s in
    tests)
      $T 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1 \
        || { tail -40 "$O/gpu_tests.log"; exit 1; }
      tail -1 "$O/gpu_tests.log" ;;
    smoke)
      $T 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 || { cat "$O/smoke.txt"; exit 1; }
      cat "$O/smoke.txt" ;;
    bench1)
      $T 300 python bench.py --inflight 1 --no-cpu-baseline > "$O/bench_inflight1.json" 2> "$O/bench1.err" \
        || { tail -20 "$O/bench1.err"; exit 1; }
      cut -c1-400 "$O/bench_inflight1.json" ;;
    bench2)
      $T 300 python bench.py > "$O/bench.json" 2> "$O/bench2.err" || { tail -20 "$O/bench2.err"; exit 1; }
      cut -c1-400 "$O/bench.json" ;;
    prof)
      (cd /tmp && $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_if1" -o trace -- \
        python "$R/bench.py" --inflight 1 --no-cpu-baseline > "$R/$O/bench_under_rocprof_inflight1.json" \
        2> "$R/$O/prof_if1.err") || { tail -20 "$O/prof_if1.err"; exit 1; }
      find "$O/prof_if1" -name "*kernel_stats.csv" -exec cut -c1-220 {} \; | head -5 ;;
    prof2)
      (cd /tmp && $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_if2" -o trace -- \
        python "$R/bench.py" --no-cpu-baseline > "$R/$O/bench_under_rocprof.json" 2> "$R/$O/prof_if2.err") \
        || { tail -20 "$O/prof_if2.err"; exit 1; }
      find "$O/prof_if2" -name "*kernel_stats.csv" -exec cut -c1-220 {} \; | head -5 ;;
    pmcwait|pmcinst|pmcmix|pmcvalu|pmcbusy|pmcic|pmcic2|pmclds)
      case $s in
        pmcbusy) C="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_IFETCH SQ_IFETCH_LEVEL GRBM_GUI_ACTIVE" ;;
        pmcic) C="SQC_ICACHE_HITS SQC_ICACHE_MISSES" ;;
        pmcic2) C="SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ" ;;
        pmclds) C="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS" ;;
        pmcwait) C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" ;;
        pmcinst) C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT" ;;
        pmcmix) C="SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT" ;;
        pmcvalu) C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F SQ_INSTS_VALU_MUL_F SQ_INSTS_VALU_FMA_F SQ_INSTS_VALU_TRANS_F SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT" ;;
      esac
      (cd /tmp && $T 120 rocprofv3 --pmc $C --output-format csv -d "$R/$O/$s/p0" -o pmc -- $(fwd) > /dev/null \
        2> "$R/$O/$s.err") || { tail -20 "$O/$s.err"; exit 1; }
      python tools/pmc_summary.py "$O/$s" informer_forward_v4 | tee "$O/$s.txt" ;;
    traffic)
      (cd /tmp && $T 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/traffic/pmc_fetch" -o pmc -- $(fwd) \
        > /dev/null 2> "$R/$O/traffic0.err") || exit 1
      (cd /tmp && $T 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/traffic/pmc_write" -o pmc -- $(fwd) \
        > /dev/null 2> "$R/$O/traffic1.err") || exit 1
      python tools/pmc_traffic.py "$O/traffic" -o "$O/pmc_traffic.json" && cat "$O/pmc_traffic.json" ;;
    stamps)
      $T 200 python tools/stamps.py 512 > "$O/stamps_b512.txt" 2> "$O/stamps.err" || { tail -20 "$O/stamps.err"; exit 1; }
      cat "$O/stamps_b512.txt" ;;
    stampsc2)
      CET_LIB=$R/channelestimationtransformer_amd/libcet_c2st.so $T 200 python tools/stamps.py 512 \
        > "$O/stamps_c2_b512.txt" 2> "$O/stampsc2.err" || { tail -20 "$O/stampsc2.err"; exit 1; }
      cat "$O/stamps_c2_b512.txt" ;;
    configs)
      $T 600 python tools/bench_configs.py > "$O/configs.jsonl" 2> "$O/configs.err" || { tail -5 "$O/configs.err"; exit 1; }
      cut -c1-300 "$O/configs.jsonl" ;;
    list)
      (cd /tmp && $T 60 rocprofv3 -L > "$R/$O/counters.txt" 2>&1) || true
      wc -l "$O/counters.txt" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
