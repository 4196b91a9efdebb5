#!/bin/bash
# rocprofv3 kernel trace of a short bench run + the per-kernel table:
#   gpu_prof.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r3}; shift || true
OUT=gpurun_out/${TAG}/trace
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-recompute --no-ref "$@" \
    > "$OUT/bench.json" 2> "$OUT/trace.log" || { echo "trace failed"; tail -20 "$OUT/trace.log"; exit 1; }
cat "$OUT/bench.json"
python3 dev/trace_table.py "$OUT" 28 > "gpurun_out/${TAG}/table.txt"
head -40 "gpurun_out/${TAG}/table.txt"
cp "$OUT"/*kernel_stats.csv "gpurun_out/${TAG}/kernel_stats.csv" 2>/dev/null
# the full trace is kept only when small enough for gpurun to copy back
find "$OUT" -name "*kernel_trace.csv" -size +40M -delete
