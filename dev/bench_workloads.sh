#!/bin/bash
# bench.py over the three single-GPU workloads (lidar = the headline line,
# fusion = configs[2], coop = configs[3] forward leg), one JSON line each.
#   gpurun --timeout 900 -- bash dev/bench_workloads.sh r1f
set -euo pipefail
TAG=${1:-r1}
OUT=gpurun_out/${TAG}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for w in lidar fusion coop; do
    timeout -k 10 300 python -u bench.py --workload $w --cpu-seconds 15 > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.log" \
        || { echo "bench $w failed"; tail -20 "$OUT/bench_$w.log"; exit 1; }
    cat "$OUT/bench_$w.json"
done
