#!/bin/bash
# Round-5 step ac: kvproj_x3 with the prologue's vmcnt(0) visible to the compiler's wait pass
# (256; the inline-asm form left a full drain at every plane's first MFMA), with the plane
# drained before its stores (128), both (384) -- alone, parity of the kv tests, bench A/B.
set -uo pipefail
TAG=${1:-r5ac}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in kv256 kv384 kvd; do
    CMT_HIP_LIB=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_split.py \
        -m gpu -q -x -k "kv or headsplit" --timeout 100 --timeout-method thread > "$OUT/tests_$v.log" 2>&1
    rc=$?; echo "$v $(tail -1 "$OUT/tests_$v.log")"; [[ $rc -eq 0 ]] || exit 1
done
for i in 1 2; do
    for v in base kvd kv256 kv384; do
        lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v != base ]] && lib=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_$v.so
        CMT_HIP_LIB=$lib timeout -k 10 60 python dev/kernel_probe.py kv --time 2>&1 | grep "per launch" | sed "s/^/$v /"
    done
done
for i in 1 2; do
    for v in base kv384; do
        lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v != base ]] && lib=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_$v.so
        CMT_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ref --no-traffic --no-recompute --steps 100 \
            > "$OUT/bench_${v}_$i.json" 2> "$OUT/bench_${v}_$i.log" || { echo "bench $v failed"; tail -20 "$OUT/bench_${v}_$i.log"; exit 1; }
        echo "$v $(python -c "import json; d=json.load(open('$OUT/bench_${v}_$i.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms')")"
    done
done
