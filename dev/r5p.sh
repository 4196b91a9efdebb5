#!/bin/bash
# Round-5 step p: kvproj_x3 K/V stores non-temporal (CMT_KV_NT=1) vs plain.
set -uo pipefail
TAG=${1:-r5p}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
NT=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_nt.so
CMT_HIP_LIB=$NT timeout -k 10 200 python -u -m pytest tests/test_gpu_split.py -m gpu -q -x -k "kv" --timeout 100 \
    --timeout-method thread > "$OUT/tests_nt.log" 2>&1; rc=$?; tail -1 "$OUT/tests_nt.log"; [[ $rc -eq 0 ]] || exit 1
for i in 1 2; do
    for v in base nt; do
        lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v == nt ]] && lib=$NT
        CMT_HIP_LIB=$lib timeout -k 10 60 python dev/kernel_probe.py kv --time 2>&1 | grep "per launch" | sed "s/^/$v /"
    done
done
for v in nt base nt base; do
    lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v == nt ]] && lib=$NT
    CMT_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ref --no-traffic --no-recompute --steps 50 \
        > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench $v failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    echo "$v $(python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms')")"
done
