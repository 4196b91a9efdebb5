#!/bin/bash
# One GPU-box pass (run from the repo root under gpurun): GPU parity tests,
# smoke(), the default bench line, then the rocprofv3 kernel-trace/stats pass
# and the FETCH_SIZE / WRITE_SIZE PMC passes (separate runs, guide rule).
# Every GPU step has its own time limit; the first failure ends the script.
#   gpurun --timeout 1100 -- bash cmt-cooperative-perception_amd/tools/gpu_check.sh r1 [tests|bench|prof|all]
set -euo pipefail
TAG=${1:-r1}
WHAT=${2:-all}
OUT=gpurun_out/${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"

if [[ $WHAT == all || $WHAT == tests ]]; then
    timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
    tail -3 "$OUT/pytest_gpu.log"
    timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
    cat "$OUT/smoke.log"
fi
if [[ $WHAT == all || $WHAT == bench ]]; then
    timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log" \
        || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
    cat "$OUT/bench.json"
fi
if [[ $WHAT == all || $WHAT == prof ]]; then
    P=$OUT/prof
    mkdir -p "$P"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$P/trace" -o run --output-format csv -- \
        python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$P/bench_trace.json" 2> "$P/trace.log" \
        || { echo "trace pass failed"; tail -20 "$P/trace.log"; exit 1; }
    timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$P/fetch" -o run -- \
        python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-graph > "$P/bench_fetch.json" 2> "$P/fetch.log" \
        || { echo "fetch pass failed"; tail -20 "$P/fetch.log"; exit 1; }
    timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$P/write" -o run -- \
        python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-graph > "$P/bench_write.json" 2> "$P/write.log" \
        || { echo "write pass failed"; tail -20 "$P/write.log"; exit 1; }
    echo "profiles done"
fi
