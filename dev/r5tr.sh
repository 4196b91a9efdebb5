#!/bin/bash
# Round-5: kernel table of the coop training step (rocprofv3 kernel trace of bench.py --train).
set -uo pipefail
TAG=${1:-r5tr}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --train --workload coop --steps 10 --warmup 3 > "$OUT/train.json" 2> "$OUT/train.log" \
    || { echo "trace failed"; tail "$OUT/train.log"; exit 1; }
python3 dev/trace_table.py "$OUT/trace" 13 > "$OUT/table.txt" 2>&1 || true
head -40 "$OUT/table.txt"
find "$OUT/trace" -name "*kernel_trace.csv" -delete
