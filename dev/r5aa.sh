#!/bin/bash
# Round-5 step aa: conv_halo_x3 with 16-byte halo loads (CMT_CONV_VAR=32) vs 4-byte loads.
set -uo pipefail
TAG=${1:-r5aa}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
QV=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_qv.so
CMT_HIP_LIB=$QV timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_head.py -m gpu -q -x -k "conv or nchw or parity or selections" \
    --timeout 200 --timeout-method thread > "$OUT/tests_qv.log" 2>&1; rc=$?; tail -1 "$OUT/tests_qv.log"
[[ $rc -eq 0 ]] || { grep -E "^FAILED|assert" "$OUT/tests_qv.log" | head; exit 1; }
for i in 1 2; do
    for v in base qv; do
        lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v == qv ]] && lib=$QV
        CMT_HIP_LIB=$lib timeout -k 10 60 python dev/kernel_probe.py convh --time 2>&1 | grep "per launch" | sed "s/^/$v /"
    done
done
for v in qv base qv base; do
    lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v == qv ]] && lib=$QV
    CMT_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ref --no-traffic --no-recompute --steps 50 \
        > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench $v failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    echo "$v $(python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms')")"
done
