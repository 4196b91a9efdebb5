#!/bin/bash
# Round-5 step r: kvproj_x3 epilogue without per-half selects (one permlane32 swap per dword,
# X as vdst / Y as vsrc) and key norms by v_dot2 -- tests, kv alone, bench, vs the previous tree.
set -uo pipefail
TAG=${1:-r5r}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
OLD=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_old.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 200 \
    --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?; tail -2 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|assert" "$OUT/tests.log" | head; exit 1; }
grep "configs\[2\] fusion.*'ref'" "$OUT/tests.log" | head -3
for i in 1 2; do
    for v in new old; do
        lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v == old ]] && lib=$OLD
        CMT_HIP_LIB=$lib timeout -k 10 60 python dev/kernel_probe.py kv --time 2>&1 | grep "per launch" | sed "s/^/$v /"
    done
done
for v in new old new old; do
    lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v == old ]] && lib=$OLD
    CMT_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ref --no-traffic --no-recompute --steps 50 \
        > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench $v failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    echo "$v $(python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms')")"
done
