#!/bin/bash
# One GPU-box pass (run from the repo root under gpurun): GPU parity tests,
# smoke(), the rocprofv3 kernel-trace/stats pass and the FETCH_SIZE /
# WRITE_SIZE PMC passes (separate runs, guide rule) of the bench workload,
# the traffic summary bench.py reads, then the bench line itself.
# Every GPU step has its own time limit; the first failure ends the script.
#   gpurun --timeout 1100 -- bash dev/gpu_check.sh r2a [tests|prof|bench|all] [workload]
set -euo pipefail
TAG=${1:-r2}
WHAT=${2:-all}
WL=${3:-fusion}
OUT=gpurun_out/${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
declare -A NK=([fusion]=56400 [lidar]=32400 [coop]=40400 [stress4]=48400)

if [[ $WHAT == all || $WHAT == tests ]]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -rA \
        > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -60 "$OUT/pytest_gpu.log"; exit 1; }
    tail -3 "$OUT/pytest_gpu.log"
    timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
    cat "$OUT/smoke.log"
fi
if [[ $WHAT == all || $WHAT == prof ]]; then
    P=$OUT/prof_$WL
    mkdir -p "$P"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$P/trace" -o run --output-format csv -- \
        python3 bench.py --workload $WL --steps 20 --warmup 5 --no-cpu-baseline --no-ref --no-traffic --no-recompute \
        > "$P/bench_trace.json" 2> "$P/trace.log" || { echo "trace pass failed"; tail -20 "$P/trace.log"; exit 1; }
    timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$P/fetch" -o run -- \
        python3 bench.py --workload $WL --steps 5 --warmup 2 --no-cpu-baseline --no-ref --no-traffic --no-graph --no-recompute \
        > "$P/bench_fetch.json" 2> "$P/fetch.log" || { echo "fetch pass failed"; tail -20 "$P/fetch.log"; exit 1; }
    timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$P/write" -o run -- \
        python3 bench.py --workload $WL --steps 5 --warmup 2 --no-cpu-baseline --no-ref --no-traffic --no-graph --no-recompute \
        > "$P/bench_write.json" 2> "$P/write.log" || { echo "write pass failed"; tail -20 "$P/write.log"; exit 1; }
    python3 dev/traffic_summary.py "$P" --tag "$TAG" --workload $WL \
        --nk ${NK[$WL]} --outdir "$P" > "$P/traffic.txt" 2>&1 || { echo "traffic summary failed"; cat "$P/traffic.txt"; exit 1; }
    mkdir -p profiles && cp "$P/${TAG}_${WL}_attn_pmc_summary.json" profiles/
    echo "profiles done"; cat "$P/traffic.txt"
fi
if [[ $WHAT == all || $WHAT == bench ]]; then
    timeout -k 10 400 python -u bench.py --workload $WL > "$OUT/bench_$WL.json" 2> "$OUT/bench_$WL.log" \
        || { echo "bench failed"; tail -20 "$OUT/bench_$WL.log"; exit 1; }
    cat "$OUT/bench_$WL.json"
fi
