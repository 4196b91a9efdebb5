#!/bin/bash
# Experiment libraries (dev only, never loaded by the product path): rebuild ONE source with
# extra -D defines and link it with the product objects into lib/exp/libcmt_hip_<tag>.so.
# Select one at run time with CMT_HIP_LIB=<path> (native.py).
#   bash dev/build_exp.sh <tag> <source.hip> "-DCMT_KV_SCHED=16 ..."   (dev-only defines: CMT_KV_SCHED, CMT_CONV_VAR, CMT_MLP_DIAG)
set -euo pipefail
TAG=$1; SRC=$2; DEFS=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/cmt-cooperative-perception_amd/csrc
LIB=$ROOT/cmt-cooperative-perception_amd/lib
make -s -C "$CS" -j8 >/dev/null
mkdir -p "$LIB/exp"
base=$(basename "$SRC" .hip)
extra=""
[[ $base == attention ]] && extra="-fno-honor-nans"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $extra $DEFS \
    -c "$CS/$base.hip" -o "$LIB/exp/${base}_$TAG.o" 2>&1 | grep -v "warning\|note:\|^ *[0-9]* | \|^ *| \|~\|\^" || true
objs=$(ls "$LIB"/obj/*.o | grep -v "/$base.o$")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$LIB/exp/libcmt_hip_$TAG.so" $objs "$LIB/exp/${base}_$TAG.o"
echo "$LIB/exp/libcmt_hip_$TAG.so"
