#!/bin/bash
# Round-4 step j: kvproj wide stores, asm halo loads in the NCHW conv, unscaled-Q cross-attention
# (tests, kernel A/B, full-size parity with both, frame A/B).
set -uo pipefail
TAG=${1:-r4j}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 250 python -u -m pytest tests/test_gpu_split.py -v -k "pipelined or f16_long or kvproj or conv3x3_nchw" \
    --timeout 150 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "tests rc=$rc"; tail -30 "$OUT/tests.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests.log" | tail -1
CMT_CONV_VAR=16 timeout -k 10 200 python -u -m pytest tests/test_gpu_split.py -v -k "conv3x3_nchw" \
    --timeout 150 --timeout-method thread > "$OUT/tests_ah.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "ah tests rc=$rc"; tail -30 "$OUT/tests_ah.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests_ah.log" | tail -1
for v in 0 64 0 64; do
    echo -n "kv sched $v: " >> "$OUT/kv.txt"
    CMT_KV_SCHED=$v timeout -k 10 120 python -u dev/kernel_probe.py kv --time 2>/dev/null | grep kv >> "$OUT/kv.txt" \
        || { echo "kv probe failed"; exit 1; }
done
cat "$OUT/kv.txt"
for v in 16 0 16 0; do
    echo -n "conv var $v: " >> "$OUT/conv.txt"
    CMT_CONV_VAR=$v timeout -k 10 120 python -u dev/kernel_probe.py convh --time 2>/dev/null | grep convh >> "$OUT/conv.txt" \
        || { echo "conv probe failed"; exit 1; }
done
cat "$OUT/conv.txt"
for v in 1 0 1 0; do
    env CMT_ATTN_US=$v CMT_ATTN_VARIANT=us$v timeout -k 10 120 python -u dev/attn_exp.py --dtype f16 --nk 56400 --bound \
        --round --qs 2>/dev/null | grep attn >> "$OUT/attn.txt" || { echo "attn_exp failed"; exit 1; }
done
cat "$OUT/attn.txt"
CMT_ATTN_US=1 CMT_CONV_VAR=16 timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py -v -rA --timeout 200 \
    --timeout-method thread > "$OUT/fullsize.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "fullsize rc=$rc"; tail -30 "$OUT/fullsize.log"; exit 1; }
grep -E "passed|failed" "$OUT/fullsize.log" | tail -1
for v in new old new old; do
    if [[ $v == new ]]; then e="CMT_ATTN_US=1 CMT_CONV_VAR=16"; else e="CMT_ATTN_US=0 CMT_CONV_VAR=0"; fi
    env $e timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-ref --no-traffic \
        --no-recompute > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" | tee -a "$OUT/bench.txt"
done
