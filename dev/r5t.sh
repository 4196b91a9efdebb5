#!/bin/bash
# Round-5 step o: what bounds kvproj_x3 -- diagnostic schedules (wrong results, timing only):
# 16 no K/V stores, 20 + no W loads, 28 + no A fragment reads.
set -uo pipefail
TAG=${1:-r5t}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_split.py -m gpu -q -x -k "kv or headsplit" --timeout 100 --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?; tail -1 "$OUT/tests.log"; [[ $rc -eq 0 ]] || exit 1
for i in 1 2; do
    for v in base old kv16 kv28; do
        lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v != base ]] && lib=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_$v.so
        CMT_HIP_LIB=$lib timeout -k 10 60 python dev/kernel_probe.py kv --time 2>&1 | grep "per launch" | sed "s/^/$v /"
    done
done
