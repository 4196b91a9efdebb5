#!/bin/bash
# Round-5 step f: issue probe with the K/V DMA stream variants; the short attention kernels'
# fp32 row sums (golden fixtures, attention tests); kvproj persistent vs one-workgroup-per-tile.
set -uo pipefail
TAG=${1:-r5f}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 ./dev/issue_probe > "$OUT/issue_probe.txt" 2>&1 || { echo "probe failed"; cat "$OUT/issue_probe.txt"; exit 1; }
grep -E "lds|dma" "$OUT/issue_probe.txt"
timeout -k 10 400 python -u -m pytest tests/test_golden.py tests/test_gpu_kernels.py tests/test_gpu_split.py tests/test_gpu_head.py -m gpu -q \
    --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -8 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error" "$OUT/tests.log" | head -20; }
LDR=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_ldr.so
CMT_HIP_LIB=$LDR timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_kernels.py -m gpu -x -q \
    -k "attention or attn" --timeout 200 --timeout-method thread > "$OUT/tests_ldr.log" 2>&1
rc=$?; tail -2 "$OUT/tests_ldr.log"
if [[ $rc -eq 0 ]]; then
    for v in base ldr base ldr; do
        lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v == ldr ]] && lib=$LDR
        CMT_HIP_LIB=$lib timeout -k 10 120 python -u dev/attn_exp.py --dtype f16 --nk 56400 --bound --qs --round --check --tag $v \
            >> "$OUT/attn.txt" 2>&1 || { echo "attn_exp $v failed"; tail -20 "$OUT/attn.txt"; exit 1; }
    done
    grep attn "$OUT/attn.txt"
else
    grep -E "^FAILED|Error" "$OUT/tests_ldr.log" | head
fi
OLD=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_kvold.so
for i in 1 2; do
    timeout -k 10 60 python dev/kernel_probe.py kv --time | grep "per launch" | sed 's/^/persistent /'
    CMT_HIP_LIB=$OLD timeout -k 10 60 python dev/kernel_probe.py kv --time | grep "per launch" | sed 's/^/per-tile   /'
done
for v in base old base old; do
    lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v == old ]] && lib=$OLD
    CMT_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ref --no-traffic --no-recompute --steps 40 \
        > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench $v failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    echo "$v $(python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms')")"
done
