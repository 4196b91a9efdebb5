#!/bin/bash
# Round-4 step k: kvproj wide stores with the corrected lane-pair swap (tests, kernel A/B,
# full-size parity at the defaults, frame A/B against the 8-byte stores), then a kernel trace.
set -uo pipefail
TAG=${1:-r4k}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 250 python -u -m pytest tests/test_gpu_split.py -v -k "kvproj" \
    --timeout 150 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "tests rc=$rc"; tail -30 "$OUT/tests.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests.log" | tail -1
for v in 0 64 0 64; do
    echo -n "kv sched $v: " >> "$OUT/kv.txt"
    CMT_KV_SCHED=$v timeout -k 10 120 python -u dev/kernel_probe.py kv --time 2>/dev/null | grep kv >> "$OUT/kv.txt" \
        || { echo "kv probe failed"; exit 1; }
done
cat "$OUT/kv.txt"
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py -v -rA --timeout 200 \
    --timeout-method thread > "$OUT/fullsize.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "fullsize rc=$rc"; tail -30 "$OUT/fullsize.log"; exit 1; }
grep -E "passed|failed" "$OUT/fullsize.log" | tail -1
for v in 0 64 0 64; do
    CMT_KV_SCHED=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-ref --no-traffic \
        --no-recompute > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('kv$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" | tee -a "$OUT/bench.txt"
done
mkdir -p "$OUT/trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref --no-traffic --no-recompute \
    > "$OUT/trace/bench.json" 2> "$OUT/trace/trace.log" || { echo "trace failed"; tail -20 "$OUT/trace/trace.log"; exit 1; }
echo done
