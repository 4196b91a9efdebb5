#!/bin/bash
# One GPU pass: a pytest selection (-k), then alternating A/B bench rounds.
#   gpurun --timeout 900 -- bash dev/ab_test.sh TAG "PYTEST_K" ROUNDS "VAR=1" "VAR=0" ...
set -euo pipefail
TAG=${1:-ab}; K=${2:-head}; ROUNDS=${3:-2}; shift 3
OUT=gpurun_out/${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s -k "$K" --timeout 150 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
bash dev/ab_bench.sh "$TAG" "$ROUNDS" "$@"
