#!/bin/bash
# Round-5 step ak: where the training step's GPU idles (kernel trace of bench.py --train, graphed
# decoder on / off).
set -uo pipefail
TAG=${1:-r5ak}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for g in 1 0; do
    CMT_TRAIN_GRAPH=$g timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/trace$g" -o run --output-format csv -- \
        python3 bench.py --train --workload coop --steps 8 --warmup 3 > "$OUT/train$g.json" 2> "$OUT/train$g.log" \
        || { echo "trace failed"; tail "$OUT/train$g.log"; exit 1; }
    echo "== graph $g"
    python3 dev/train_gaps.py "$OUT/trace$g" 2>&1 | tee "$OUT/gaps$g.txt"
    find "$OUT/trace$g" -name "*kernel_trace.csv" -delete
done
