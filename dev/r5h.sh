#!/bin/bash
# Round-5 step h: golden fixtures + attention tests with the exact row-maximum pre-pass.
set -uo pipefail
TAG=${1:-r5h}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_golden.py tests/test_gpu_kernels.py tests/test_gpu_split.py -m gpu -q \
    --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -12 "$OUT/tests.log"; exit $rc
