#!/bin/bash
# Training-step evidence pass (GPU box): the configs[3] head training bench and
# its kernel trace.  gpu_train.sh <tag>
set -o pipefail
TAG=${1:-r3t}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --train --workload coop --steps 50 --warmup 5 > "$OUT/train.json" 2> "$OUT/train.log" || { tail -5 "$OUT/train.log"; exit 1; }
cat "$OUT/train.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/train_trace" -o run --output-format csv -- \
    python3 bench.py --train --workload coop --steps 20 --warmup 3 > "$OUT/train_trace.json" 2> "$OUT/train_trace.log" || { echo "trace failed"; exit 1; }
python3 dev/trace_table.py "$OUT/train_trace" 23 > "$OUT/train_table.txt"
head -30 "$OUT/train_table.txt"
cp "$OUT"/train_trace/*kernel_stats.csv "$OUT/train_kernel_stats.csv" 2>/dev/null
rm -rf "$OUT/train_trace"
