#!/bin/bash
# Build an A/B copy of the engine library from the committed HEAD (working-tree changes stashed):
#   tools/build_ab.sh [NAME]   -> channelestimationtransformer_amd/libcet_NAME.so (default NAME=base)
# (EXTRA in the environment: extra compiler flags, e.g. EXTRA=-DCET_C2_STAMPS)
set -e
NAME=${1:-base}
cd "$(dirname "$0")/.."
git stash -q
trap 'git stash pop -q' EXIT
make -C channelestimationtransformer_amd/csrc -j8 OUT=../libcet_$NAME.so B=build_$NAME EXTRA="$EXTRA" > /tmp/mk_$NAME.log 2>&1
