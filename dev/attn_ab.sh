#!/bin/bash
# Cross-attention A/B on the GPU box: one pytest selection, then the attention
# microbenchmark (fusion shape, bounded mode) and the bench line per env variant.
#   gpurun --timeout 600 -- bash dev/attn_ab.sh TAG "PYTEST_K" ["ENV=1" ...]
set -euo pipefail
TAG=${1:-ab}
K=${2:-attention}
shift 2 || true
OUT=gpurun_out/${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s -k "$K" --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
grep -E "passed|failed|max rel" "$OUT/pytest_gpu.log" | tail -12
i=0
for variant in "" "$@"; do
    i=$((i + 1))
    env $variant timeout -k 10 120 python -u dev/attn_exp.py --nk 56400 --bound \
        --check --tag "v$i:$variant" >> "$OUT/attn.txt" 2>&1 || { echo "attn_exp [$variant] failed"; tail -20 "$OUT/attn.txt"; exit 1; }
    env $variant timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ref --no-traffic --no-recompute > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.log" \
        || { echo "bench [$variant] failed"; tail -20 "$OUT/bench_$i.log"; exit 1; }
    echo "[$variant] $(python -c "import json,sys; d=json.load(open('$OUT/bench_$i.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms', 'attn', d['roofline']['avg_launch_ms'], 'ms', d['roofline']['frac'])")"
done
cat "$OUT/attn.txt"
