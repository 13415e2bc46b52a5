#!/bin/bash
# Per-phase stamps of several C2-stamps builds on one box, alternated twice:
#   tools/stamps_ab.sh OUTDIR LIB [LIB ...]   (each LIB built with -DCET_C2_STAMPS)
cd "$GRAFT_REPO_ROOT"
O=$1; shift
mkdir -p "$O"
for i in 1 2; do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    CET_LIB=$(pwd)/$lib timeout -k 10 200 python tools/stamps.py 512 > "$O/${n}_$i.txt" 2> "$O/${n}_$i.err" || exit 1
    echo "$n $i: $(sed -n 2p "$O/${n}_$i.txt")"
  done
done
