#!/bin/bash
# One GPU-box pass of round-3 checks: gpu_r3.sh <tag> "<pytest targets>" [bench args | none]
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
TAG=${1:-r3}
TESTS=${2:-tests/test_gpu_split.py}
BENCH=${3:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [[ "$TESTS" != none ]]; then
    timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread -rA > "$OUT/pytest.log" 2>&1
    rc=$?
    grep -E "^(PASSED|FAILED|ERROR)|passed|failed|^E  " "$OUT/pytest.log" | tail -40
    sed -n '/measured parity/,$p' "$OUT/pytest.log" | head -30
    [ $rc -eq 0 ] || exit $rc
fi
if [[ -n "$BENCH" && "$BENCH" != none ]]; then
    timeout -k 10 400 python -u bench.py $BENCH > "$OUT/bench.json" 2> "$OUT/bench.log"
    rc=$?
    cat "$OUT/bench.json"; tail -3 "$OUT/bench.log"
    exit $rc
fi
