#!/bin/bash
# Final evidence of a round on the final tree: full GPU suite (parity lines -> r5_parity), smoke,
# rocprofv3 kernel trace + stats of the default bench, one 'ref' frame's timeline, FETCH_SIZE and
# WRITE_SIZE passes (separate; the roofline form: split combine as its own launch), the default
# bench line and the coop training bench.
set -uo pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error" "$OUT/tests.log" | head -20; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-ref > "$OUT/bench_trace.json" 2> "$OUT/trace.log" \
    || { echo "trace failed"; tail "$OUT/trace.log"; exit 1; }
python3 dev/timeline.py "$OUT/trace" 8 > "$OUT/frame_timeline.txt" 2>&1 || true
tail -1 "$OUT/frame_timeline.txt"
python3 dev/trace_table.py "$OUT/trace" > "$OUT/kernel_table.txt" 2>&1 || true
CMT_CHAIN_COMBINE=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof/fetch" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-graph --no-traffic --no-ref --no-recompute > "$OUT/bench_fetch.json" 2> "$OUT/fetch.log" \
    || { echo "fetch pass failed"; tail "$OUT/fetch.log"; exit 1; }
CMT_CHAIN_COMBINE=0 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/prof/write" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-graph --no-traffic --no-ref --no-recompute > "$OUT/bench_write.json" 2> "$OUT/write.log" \
    || { echo "write pass failed"; tail "$OUT/write.log"; exit 1; }
python3 dev/traffic_summary.py "$OUT/prof" --tag "$TAG" --workload fusion --nk 56400 --outdir "$OUT" > "$OUT/traffic.txt" 2>&1 \
    || { cat "$OUT/traffic.txt"; exit 1; }
find "$OUT/prof" -name "*.db" -delete
cp "$OUT/${TAG}_fusion_attn_pmc_summary.json" profiles/ 2>/dev/null
timeout -k 10 400 python3 -u bench.py > "$OUT/bench_fusion.json" 2> "$OUT/bench_fusion.log" \
    || { echo "bench failed"; tail "$OUT/bench_fusion.log"; exit 1; }
cat "$OUT/bench_fusion.json"
timeout -k 10 400 python3 -u bench.py --train --workload coop > "$OUT/train_coop.json" 2> "$OUT/train_coop.log" \
    || { echo "train bench failed"; tail "$OUT/train_coop.log"; exit 1; }
cat "$OUT/train_coop.json"
