#!/bin/bash
# Round-4 step z16: cmt_mlp2_x3 with two waves per SIMD (OS = 2: 8 waves, each half of the output
# tiles, fc1 computed by both waves of a row group) vs one (OS = 1): mlp tests both ways, kernel
# probe, full-size fusion parity with OS = 2, frame A/B alternating.
set -uo pipefail
TAG=${1:-r4z16}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 2 1; do
    CMT_MLP_OS=$v timeout -k 10 200 python -u -m pytest tests/test_gpu_mlp.py -q --timeout 100 --timeout-method thread \
        > "$OUT/tests_$v.log" 2>&1 || { echo "mlp tests OS=$v failed"; tail -30 "$OUT/tests_$v.log"; exit 1; }
    echo "OS=$v $(tail -1 "$OUT/tests_$v.log")"
done
for v in 2 1 2 1; do
    CMT_MLP_OS=$v timeout -k 10 200 python -u dev/mlp_probe.py > "$OUT/probe_$v.txt" 2>&1 || { echo "probe failed"; tail -20 "$OUT/probe_$v.txt"; exit 1; }
    echo "OS=$v $(grep 'M=24000' "$OUT/probe_$v.txt")"
done
CMT_MLP_OS=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -q -rA -k "fusion" --timeout 300 \
    --timeout-method thread > "$OUT/fullsize.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "fullsize rc=$rc"; tail -30 "$OUT/fullsize.log"; exit 1; }
grep -E "passed|failed" "$OUT/fullsize.log" | tail -1
for v in 2 1 2 1 2 1; do
    CMT_MLP_OS=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-ref --no-traffic \
        --no-recompute > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('os$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" | tee -a "$OUT/bench.txt"
done
echo done
