#!/bin/bash
# Round-4 step z6: bf16x3 GEMM with two 32-k sub-tiles per step: GEMM probe A/B (lib_old = HEAD),
# training kernel tests, training bench A/B.
set -uo pipefail
TAG=${1:-r4z6}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
OLD=cmt-cooperative-perception_amd/lib_old/libcmt_hip.so
for l in new old new old; do
    if [[ $l == old ]]; then export CMT_HIP_LIB=$OLD; else unset CMT_HIP_LIB; fi
    timeout -k 10 120 python -u dev/gemm_probe.py >> "$OUT/probe.txt" 2>&1 || { echo "probe failed"; tail -20 "$OUT/probe.txt"; exit 1; }
done
unset CMT_HIP_LIB
grep -v amdgpu.ids "$OUT/probe.txt"
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_kernels.py tests/test_gpu_train_head.py -v --timeout 200 \
    --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "tests rc=$rc"; tail -30 "$OUT/tests.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests.log" | tail -1
for l in new old new old; do
    if [[ $l == old ]]; then export CMT_HIP_LIB=$OLD; else unset CMT_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --train --workload coop --steps 30 --warmup 5 \
        > "$OUT/train_$l.json" 2> "$OUT/train_$l.log" || { echo "train bench failed"; tail -5 "$OUT/train_$l.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/train_$l.json'));print('$l', d['value'], d['ms_per_step'])" | tee -a "$OUT/train.txt"
done
echo done
