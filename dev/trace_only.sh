#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC):
#   gpurun -- bash dev/trace_only.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-r1}; shift || true
OUT=gpurun_out/${TAG}/trace
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/trace.log" \
    || { echo "trace failed"; tail -20 "$OUT/trace.log"; exit 1; }
cat "$OUT/bench.json"
