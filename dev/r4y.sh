#!/bin/bash
# Round-4 step y: host-side profile of the coop training step, and its kernel table with the
# prefetching bf16x3 GEMM.
set -uo pipefail
TAG=${1:-r4y}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u dev/train_host_profile.py > "$OUT/host_profile.txt" 2>&1 || { echo "profile failed"; tail -20 "$OUT/host_profile.txt"; exit 1; }
grep "ms/step" "$OUT/host_profile.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/train_trace" -o run --output-format csv -- \
    python3 bench.py --train --workload coop --steps 20 --warmup 3 > "$OUT/train_trace.json" 2> "$OUT/train_trace.log" || { echo "trace failed"; exit 1; }
python3 dev/trace_table.py "$OUT/train_trace" 23 > "$OUT/train_table.txt"
head -30 "$OUT/train_table.txt" | cut -c1-160
cp "$OUT"/train_trace/*kernel_stats.csv "$OUT/train_kernel_stats.csv" 2>/dev/null
rm -rf "$OUT/train_trace"
echo done
