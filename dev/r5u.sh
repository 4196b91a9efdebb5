#!/bin/bash
# Round-5 step u: range guard in the 128-wide split tile and the training conv; split tests.
set -uo pipefail
TAG=${1:-r5u}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_head.py tests/test_gpu_split.py tests/test_gpu_head.py -m gpu -q -x \
    --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?; tail -3 "$OUT/tests.log"
[[ $rc -eq 0 ]] || { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit 1; }
