#!/bin/bash
# Final evidence of a round on the final tree, one GPU call (each GPU step under its own limit, the
# first failure ends the script):
#   1. the full GPU suite (its parity lines) and smoke();
#   2. rocprofv3 kernel trace + stats of the default bench's headline frame (no side workloads) and
#      one 'ref' frame's timeline;
#   3. FETCH_SIZE / WRITE_SIZE passes (separate) of the same frame, eager, the cross-attention core
#      as the frame runs it (split partials for chain B1) -> profiles/<tag>_fusion_attn_pmc_summary.json;
#   4. SQ / TCC counter passes (dev/pmc_passes.sh) of the pre-attention kernels on their probes;
#   5. the default bench line (every config's side key, the CPU baseline);
#   6. the coop training step's kernel trace.
#   gpurun --timeout 1200 -- bash dev/final_evidence.sh r6z [skip-tests]
set -uo pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [[ ${2:-} != skip-tests ]]; then
    timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
    rc=$?; tail -3 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error" "$OUT/tests.log" | head -20; exit 1; }
    timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 1; }
    tail -2 "$OUT/smoke.log"
fi
NOSIDE="--no-cpu-baseline --no-traffic --no-ref --no-side --no-recompute"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 $NOSIDE > "$OUT/bench_trace.json" 2> "$OUT/trace.log" \
    || { echo "trace failed"; tail "$OUT/trace.log"; exit 1; }
python3 dev/timeline.py "$OUT/trace" 8 > "$OUT/frame_timeline.txt" 2>&1 || true
tail -1 "$OUT/frame_timeline.txt"
python3 dev/trace_table.py "$OUT/trace" > "$OUT/kernel_table.txt" 2>&1 || true
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof/fetch" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-graph $NOSIDE > "$OUT/bench_fetch.json" 2> "$OUT/fetch.log" \
    || { echo "fetch pass failed"; tail "$OUT/fetch.log"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/prof/write" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-graph $NOSIDE > "$OUT/bench_write.json" 2> "$OUT/write.log" \
    || { echo "write pass failed"; tail "$OUT/write.log"; exit 1; }
python3 dev/traffic_summary.py "$OUT/prof" --tag "$TAG" --workload fusion --nk 56400 --outdir "$OUT" \
    --match attn_pb2_kernel > "$OUT/traffic.txt" 2>&1 || { cat "$OUT/traffic.txt"; exit 1; }
find "$OUT/prof" -name "*.db" -delete
cp "$OUT/${TAG}_fusion_attn_pmc_summary.json" profiles/ 2>/dev/null
for k in convh:conv_halo kv:kvproj_x3 mlp:mlp2_x3; do
    timeout -k 10 400 bash dev/pmc_passes.sh "$OUT/pmc_${k%%:*}" "${k##*:}" dev/kernel_probe.py "${k%%:*}" --iters 5 \
        > "$OUT/pmc_${k%%:*}.txt" 2>&1 || { echo "pmc ${k%%:*} failed"; tail "$OUT/pmc_${k%%:*}.txt"; exit 1; }
done
timeout -k 10 500 python3 -u bench.py > "$OUT/bench_fusion.json" 2> "$OUT/bench_fusion.log" \
    || { echo "bench failed"; tail "$OUT/bench_fusion.log"; exit 1; }
cat "$OUT/bench_fusion.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/train_trace" -o run --output-format csv -- \
    python3 bench.py --train --workload coop --steps 20 --warmup 5 > "$OUT/train_coop.json" 2> "$OUT/train_trace.log" \
    || { echo "train trace failed"; tail "$OUT/train_trace.log"; exit 1; }
cat "$OUT/train_coop.json"
python3 dev/trace_table.py "$OUT/train_trace" 25 60 > "$OUT/train_kernel_table.txt" 2>&1 || true
find "$OUT" -name "*.db" -delete
exit 0
