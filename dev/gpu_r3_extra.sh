#!/bin/bash
# Round-3 evidence pass (GPU box): SQ counters of the ref-policy cross-attention
# launch, the training bench and its kernel trace.  gpu_r3_extra.sh <tag>
set -o pipefail
TAG=${1:-r3x}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash dev/attn_pmc.sh "$TAG/attn_ref" --dtype f16 --nk 56400 --bound --round || exit 1
timeout -k 10 300 python -u bench.py --train --steps 50 --warmup 5 > "$OUT/train.json" 2> "$OUT/train.log" || { tail -5 "$OUT/train.log"; exit 1; }
cat "$OUT/train.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/train_trace" -o run --output-format csv -- \
    python3 bench.py --train --steps 20 --warmup 3 > "$OUT/train_trace.json" 2> "$OUT/train_trace.log" || { echo "trace failed"; exit 1; }
python3 dev/trace_table.py "$OUT/train_trace" 23 > "$OUT/train_table.txt"
head -30 "$OUT/train_table.txt"
cp "$OUT"/train_trace/*kernel_stats.csv "$OUT/train_kernel_stats.csv" 2>/dev/null
rm -rf "$OUT/train_trace"
