#!/bin/bash
# Alternating A/B of bench.py env variants on one GPU box (thermal/clock drift
# averages out): ROUNDS x (each variant once), 200 timed frames per run.
#   gpurun --timeout 900 -- bash dev/ab_bench.sh TAG ROUNDS "VAR=1" "VAR=0" ...
set -euo pipefail
TAG=${1:-ab}; ROUNDS=${2:-3}; shift 2
OUT=gpurun_out/${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for r in $(seq 1 "$ROUNDS"); do
    i=0
    for variant in "$@"; do
        i=$((i + 1))
        env $variant timeout -k 10 200 python -u bench.py --steps 200 --warmup 30 --no-cpu-baseline --no-ref --no-recompute \
            --no-traffic > "$OUT/b_${r}_$i.json" 2> "$OUT/b_${r}_$i.log" || { echo "bench [$variant] failed"; tail -20 "$OUT/b_${r}_$i.log"; exit 1; }
        echo "round $r [$variant] $(python -c "import json; d=json.load(open('$OUT/b_${r}_$i.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms attn', d['roofline']['avg_launch_ms'])")"
    done
done
