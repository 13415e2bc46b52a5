#!/bin/bash
# A/B kernel timing on one box: tools/ab.sh <lib_a> <lib_b> — alternates the two builds twice
# (steady-state "resident sampler again" line of tools/ablate.py).
set -o pipefail
for i in 1 2; do
  for L in "$1" "$2"; do
    echo -n "$(basename $L): "
    CET_LIB=$L timeout -k 10 120 python tools/ablate.py 3 2>/dev/null | grep again || exit 1
  done
done
