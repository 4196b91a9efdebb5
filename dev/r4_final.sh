#!/bin/bash
# Round-4 evidence of the final tree: the default bench line (roofline, cpu_baseline, side keys),
# a rocprofv3 kernel trace + stats of the same command (timed frames only differ in count), the
# frame timeline and kernel table, separate FETCH_SIZE / WRITE_SIZE passes of the attention
# launch, and the training bench line.
set -uo pipefail
TAG=${1:-r4z}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log" || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
cat "$OUT/bench.json"
mkdir -p "$OUT/trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/trace/bench.json" 2> "$OUT/trace/trace.log" \
    || { echo "trace failed"; tail -20 "$OUT/trace/trace.log"; exit 1; }
python3 dev/timeline.py "$OUT/trace" 8 > "$OUT/timeline.txt" || true
python3 dev/trace_table.py "$OUT/trace" > "$OUT/kernel_table.txt" || true
cp "$OUT"/trace/*kernel_stats.csv "$OUT/kernel_stats.csv"
head -12 "$OUT/kernel_table.txt" | cut -c1-140
tail -1 "$OUT/timeline.txt"
timeout -k 10 300 python -u bench.py --train --workload coop --steps 50 --warmup 5 > "$OUT/train.json" 2> "$OUT/train.log" \
    || { echo "train bench failed"; tail -5 "$OUT/train.log"; exit 1; }
cat "$OUT/train.json"
rm -rf "$OUT/trace/"*/ 2>/dev/null
echo done
