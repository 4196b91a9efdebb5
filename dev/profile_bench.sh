#!/bin/bash
# rocprofv3 passes over bench.py for profiles/ (run on the GPU box from the repo root):
#   1. kernel trace + stats (per-kernel durations of a 20-step bf16 bench)
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate: they share TCC counter slots)
# Output under gpurun_out/prof_<tag>/; summarise with dev/pmc_summary.py and
# dev/traffic_summary.py.
set -euo pipefail
TAG=${1:-r1}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_trace.json" 2> "$OUT/trace.log"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-graph > "$OUT/bench_fetch.json" 2> "$OUT/fetch.log"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-graph > "$OUT/bench_write.json" 2> "$OUT/write.log"
echo done
