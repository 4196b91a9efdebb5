#!/bin/bash
# Round-4 step z15: minimum reduction rows per split-K part of the training weight-gradient GEMMs
# (CMT_KSPLIT_MIN 64 vs 256): GEMM probe, tests, training bench alternating.
set -uo pipefail
TAG=${1:-r4z15}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 64 256; do
    echo "ksplit_min $v" >> "$OUT/probe.txt"
    CMT_KSPLIT_MIN=$v timeout -k 10 120 python -u dev/gemm_probe.py >> "$OUT/probe.txt" 2>&1 || { echo "probe failed"; tail -20 "$OUT/probe.txt"; exit 1; }
done
grep -v amdgpu.ids "$OUT/probe.txt"
CMT_KSPLIT_MIN=64 timeout -k 10 400 python -u -m pytest tests/test_gpu_train_kernels.py tests/test_gpu_train_head.py -v --timeout 200 \
    --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "tests rc=$rc"; tail -30 "$OUT/tests.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests.log" | tail -1
for v in 64 256 64 256 64 256; do
    CMT_KSPLIT_MIN=$v timeout -k 10 300 python -u bench.py --train --workload coop --steps 30 --warmup 5 \
        > "$OUT/train_$v.json" 2> "$OUT/train_$v.log" || { echo "train bench failed"; tail -5 "$OUT/train_$v.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/train_$v.json'));print('ksmin$v', d['value'], d['ms_per_step'])" | tee -a "$OUT/train.txt"
done
echo done
