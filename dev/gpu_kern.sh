#!/bin/bash
# Kernel microbenchmarks under env variants (no tests):
#   gpurun --timeout 600 -- bash dev/gpu_kern.sh TAG ONLY ["ENV=1" ...]
set -euo pipefail
TAG=${1:-kern}
ONLY=${2:-chain}
shift 2 || true
OUT=gpurun_out/${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
i=0
for variant in "" "$@"; do
    i=$((i + 1))
    echo "== [$variant]"
    env $variant timeout -k 10 200 python -u dev/bench_kernels.py --only "$ONLY" \
        > "$OUT/k_$i.txt" 2>&1 || { echo "bench_kernels [$variant] failed"; tail -20 "$OUT/k_$i.txt"; exit 1; }
    grep -v amdgpu.ids "$OUT/k_$i.txt"
done
