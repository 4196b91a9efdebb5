#!/bin/bash
# Round-5 step w: the one-launch camera rows alone vs three launches; diagnostic builds
# (md1 no C2 stores, md2 no NCHW loads, md4 no coordinates, md7 none of them).
set -uo pipefail
TAG=${1:-r5w}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in base base; do
    lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v != base ]] && lib=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_$v.so
    TAG=$v CMT_HIP_LIB=$lib timeout -k 10 90 python dev/mlp_geo_probe.py 2>&1 | grep fused || { echo "$v failed"; exit 1; }
done
