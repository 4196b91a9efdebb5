#!/bin/bash
# Round-5 step aj: which gradients differ between the graphed and the op-by-op training decoder.
set -uo pipefail
TAG=${1:-r5aj}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_head.py -m gpu -v -x --timeout 200 --timeout-method thread \
    -k "graph" > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; grep -E "assert|Error" "$OUT/tests.log" | head -20
