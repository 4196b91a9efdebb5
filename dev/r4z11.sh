#!/bin/bash
# Round-4 step z11: full-size parity + head tests with the fused query-side RV MLP.
set -uo pipefail
TAG=${1:-r4z11}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_head.py tests/test_gpu_mlp.py -v -rA \
    --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "tests rc=$rc"; tail -30 "$OUT/tests.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests.log" | tail -1
grep -E "^FAILED|full-size" "$OUT/tests.log" | head -20
echo done
