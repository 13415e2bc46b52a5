#!/bin/bash
# Vector-memory-path PMC passes (L1/TA/L2 traffic and stalls) over tools/run_forward.py; one rocprofv3
# run per pass.  Outputs in gpurun_out/$1/p*/ ; summary: python tools/pmc_summary.py gpurun_out/$1
set -euo pipefail
TAG=${1:-pmc_mem}; V=${2:-4}; B=${3:-512}
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p "$O"; export TMPDIR=/tmp; cd /tmp
i=0
for grp in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" ; do
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$O/p$i" -o pmc -- python "$R/tools/run_forward.py" 10 $B $V > /dev/null 2> "$O/p$i.err"
  i=$((i+1))
done
echo done > "$O/DONE"
