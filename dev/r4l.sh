#!/bin/bash
# Round-4 step l: the one-launch rv_embedding (cmt_mlp2_x3): kernel tests, path agreement,
# kernel timing, full-size parity (fusion / coop use it), frame A/B, kernel trace.
set -uo pipefail
TAG=${1:-r4l}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_head.py -v -k "mlp or path_selections" \
    --timeout 150 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "tests rc=$rc"; tail -30 "$OUT/tests.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests.log" | tail -1
timeout -k 10 120 python -u dev/mlp_probe.py > "$OUT/mlp.txt" 2>&1 || { echo "probe failed"; tail -20 "$OUT/mlp.txt"; exit 1; }
cat "$OUT/mlp.txt"
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py -v -rA -k "fusion or coop" --timeout 200 \
    --timeout-method thread > "$OUT/fullsize.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "fullsize rc=$rc"; tail -30 "$OUT/fullsize.log"; exit 1; }
grep -E "passed|failed" "$OUT/fullsize.log" | tail -1
for v in 1 0 1 0; do
    CMT_MLP_FUSED=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-ref --no-traffic \
        --no-recompute > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('mlp_fused$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" | tee -a "$OUT/bench.txt"
done
mkdir -p "$OUT/trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref --no-traffic --no-recompute \
    > "$OUT/trace/bench.json" 2> "$OUT/trace/trace.log" || { echo "trace failed"; tail -20 "$OUT/trace/trace.log"; exit 1; }
echo done
