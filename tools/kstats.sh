#!/bin/bash
# Register / spill / LDS summary of the kernels of one translation unit (compiler view):
#   tools/kstats.sh cet_informer4_bf16.hip [extra flags]     (run from anywhere)
cd "$(dirname "$0")/../channelestimationtransformer_amd/csrc"
TU=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 --cuda-device-only -c -o /tmp/kstats.o \
  -fno-honor-nans -mllvm -amdgpu-use-amdgpu-trackers -Rpass-analysis=kernel-resource-usage "$@" "$TU" 2>&1 |
  grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|SGPRs:|LDS" | paste - - - - - - - | \
  sed 's/remark: //g; s/\[-Rpass-analysis=kernel-resource-usage\]//g' | awk '{$1=$1};1' | cut -c1-400
