#!/bin/bash
# Round-4 step z2: training step changes: kernel + head training tests, training bench x2, host profile.
# Linears with the ABI-16 bias stride, layer-invariant loss terms hoisted): kernel + head training
# tests, training bench x2, host profile.
set -uo pipefail
TAG=${1:-r4z2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_kernels.py tests/test_gpu_train_head.py -v --timeout 200 \
    --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "tests rc=$rc"; tail -30 "$OUT/tests.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests.log" | tail -1
grep -E "FAILED|Error" "$OUT/tests.log" | head -10
for l in a b; do
    timeout -k 10 300 python -u bench.py --train --workload coop --steps 30 --warmup 5 \
        > "$OUT/train_$l.json" 2> "$OUT/train_$l.log" || { echo "train bench failed"; tail -5 "$OUT/train_$l.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/train_$l.json'));print('$l', d['value'], d['ms_per_step'])" | tee -a "$OUT/train.txt"
done
timeout -k 10 300 python -u dev/train_host_profile.py > "$OUT/host_profile.txt" 2>&1 || { echo "profile failed"; tail -20 "$OUT/host_profile.txt"; exit 1; }
grep "ms/step" "$OUT/host_profile.txt"
echo done
