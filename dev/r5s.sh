#!/bin/bash
# Round-5 step s: kvproj_x3 K/V stores staged through a per-wave LDS slice (CMT_KV_STG=1:
# 1 KB contiguous per store instruction) vs two half-row pieces per lane.
set -uo pipefail
TAG=${1:-r5s}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
STG=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_stg.so
CMT_HIP_LIB=$STG timeout -k 10 200 python -u -m pytest tests/test_gpu_split.py -m gpu -q -x -k "kv or headsplit" --timeout 100 \
    --timeout-method thread > "$OUT/tests_stg.log" 2>&1; rc=$?; tail -1 "$OUT/tests_stg.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|assert" "$OUT/tests_stg.log" | head; exit 1; }
for i in 1 2; do
    for v in base stg; do
        lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v == stg ]] && lib=$STG
        CMT_HIP_LIB=$lib timeout -k 10 60 python dev/kernel_probe.py kv --time 2>&1 | grep "per launch" | sed "s/^/$v /"
    done
done
for v in stg base stg base; do
    lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v == stg ]] && lib=$STG
    CMT_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ref --no-traffic --no-recompute --steps 50 \
        > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench $v failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    echo "$v $(python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms')")"
done
