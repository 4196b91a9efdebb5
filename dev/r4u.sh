#!/bin/bash
# Round-4 step u: ping-pong attention with the DMA duty split between the halves (CMT_ATTN_VB=1):
# long-key tests with it, kernel A/B, full-size fusion parity with it, frame A/B.
set -uo pipefail
TAG=${1:-r4u}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
CMT_ATTN_VB=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -v -k "f16_long or pipelined" \
    --timeout 150 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "tests rc=$rc"; tail -30 "$OUT/tests.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests.log" | tail -1
for v in 1 0 1 0 1 0; do
    CMT_ATTN_VB=$v timeout -k 10 120 python -u dev/attn_exp.py --dtype f16 --nk 56400 --bound --round --qs 2>/dev/null \
        | grep attn | sed "s/^/vb$v /" >> "$OUT/attn.txt" || { echo "attn_exp failed"; exit 1; }
done
cat "$OUT/attn.txt"
CMT_ATTN_VB=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -v -rA -k "fusion" --timeout 200 \
    --timeout-method thread > "$OUT/fullsize.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "fullsize rc=$rc"; tail -30 "$OUT/fullsize.log"; exit 1; }
grep -E "passed|failed" "$OUT/fullsize.log" | tail -1
for v in 1 0 1 0; do
    CMT_ATTN_VB=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-ref --no-traffic \
        --no-recompute > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('vb$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" | tee -a "$OUT/bench.txt"
done
echo done
