#!/bin/bash
# Round-5 step q: kvproj_x3 with the SIMD's second wave started late (s_sleep 16 / 32 / 48 x 64 cycles).
set -uo pipefail
TAG=${1:-r5q}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do
    for v in base sl16 sl32 sl48; do
        lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v != base ]] && lib=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_$v.so
        CMT_HIP_LIB=$lib timeout -k 10 60 python dev/kernel_probe.py kv --time 2>&1 | grep "per launch" | sed "s/^/$v /"
    done
done
