#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over tools/run_forward.py; outputs in gpurun_out/$1
set -euo pipefail
TAG=${1:-pmc}; V=${2:-4}
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p "$O"; export TMPDIR=/tmp; cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_IFETCH SQ_LDS_BANK_CONFLICT" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" ; do
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$O/p$i" -o pmc -- python "$R/tools/run_forward.py" 10 512 $V > /dev/null 2> "$O/p$i.err"
  i=$((i+1))
done
echo done > "$O/DONE"
