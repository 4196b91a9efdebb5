#!/bin/bash
# GPU experiment pass: the GPU tests, then bench.py under env variants (A/B of
# kernel choices), then the attention microbenchmark.
#   gpurun --timeout 900 -- bash dev/gpu_exp.sh TAG ["ENV=1 ENV2=0" ...]
set -euo pipefail
TAG=${1:-exp}
shift || true
OUT=gpurun_out/${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
i=0
for variant in "" "$@"; do
    i=$((i + 1))
    env $variant timeout -k 10 200 python -u bench.py --no-cpu-baseline > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.log" \
        || { echo "bench [$variant] failed"; tail -20 "$OUT/bench_$i.log"; exit 1; }
    echo "[$variant] $(python -c "import json,sys; d=json.load(open('$OUT/bench_$i.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms', 'attn', d['roofline']['avg_launch_ms'], 'ms', d['roofline']['frac'])")"
done
timeout -k 10 200 python -u dev/bench_kernels.py --only attn > "$OUT/kernels_attn.txt" 2>&1 \
    || { echo "bench_kernels failed"; tail -20 "$OUT/kernels_attn.txt"; exit 1; }
cat "$OUT/kernels_attn.txt"
