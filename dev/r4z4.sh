#!/bin/bash
# Round-4 step z4: coop training kernel table and GPU busy fraction / idle gaps of the step.
set -uo pipefail
TAG=${1:-r4z4}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/train_trace" -o run --output-format csv -- \
    python3 bench.py --train --workload coop --steps 20 --warmup 3 > "$OUT/train_trace.json" 2> "$OUT/train_trace.log" || { echo "trace failed"; exit 1; }
python3 dev/trace_table.py "$OUT/train_trace" 23 > "$OUT/train_table.txt"
python3 dev/trace_busy.py "$OUT/train_trace" 0.8 > "$OUT/train_busy.txt"
cat "$OUT/train_busy.txt"
head -30 "$OUT/train_table.txt" | cut -c1-160
cp "$OUT"/train_trace/*kernel_stats.csv "$OUT/train_kernel_stats.csv" 2>/dev/null
rm -rf "$OUT/train_trace"
echo done
