#!/bin/bash
# Round-4 step z19: BatchNorm sums back on 256-row blocks (deterministic order), loop unrolled:
# the DP gradient-exchange test, training tests, kernel time.
set -uo pipefail
TAG=${1:-r4z19}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_0_dp_train.py tests/test_gpu_train_kernels.py tests/test_gpu_train_head.py \
    -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed" "$OUT/tests.log" | tail -1; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error" "$OUT/tests.log" | head; exit 1; }
bash dev/r4z4.sh "${TAG}t" > /dev/null 2>&1 || { echo "trace failed"; exit 1; }
grep -E "bn_bwd_sums|col_sum" "gpurun_out/${TAG}t/train_kernel_stats.csv" | cut -c1-160
echo done
