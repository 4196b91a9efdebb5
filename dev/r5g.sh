#!/bin/bash
# Round-5 step g: the pruned library (tile-at-a-time kernel, priorities and the persistent kv
# projection removed) and the exact row-maximum pre-pass of the short f16 cross-attention core:
# the full GPU suite (golden logits every layer <= 1e-3), then a bench run.
set -uo pipefail
TAG=${1:-r5g}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -4 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error" "$OUT/tests.log" | head -20; exit 1; }
grep -i "golden" "$OUT/tests.log" | head -10
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ref --no-traffic --no-recompute --steps 40 \
    > "$OUT/bench.json" 2> "$OUT/bench.log" || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
cat "$OUT/bench.json"
