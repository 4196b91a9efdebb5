#!/bin/bash
# Round-4 step i: kvproj epilogue diagnostics, the pipelined/ping-pong attention test, and a
# kernel trace of the bench (frame timeline with the split chains).
set -uo pipefail
TAG=${1:-r4i}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_split.py -v -k "pipelined or f16_long or kvproj" \
    --timeout 150 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
[[ $rc -eq 0 || $rc -eq 1 ]] || { echo "tests rc=$rc"; tail -30 "$OUT/tests.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests.log" | tail -2
for v in ${KV_VARIANTS:-0 16 32 48 60 13 0 16 32}; do
    echo -n "kv sched $v: " >> "$OUT/kv.txt"
    CMT_KV_SCHED=$v timeout -k 10 120 python -u dev/kernel_probe.py kv --time 2>/dev/null >> "$OUT/kv.txt" \
        || { echo "kv probe failed"; tail -5 "$OUT/kv.txt"; exit 1; }
done
grep "kv sched" "$OUT/kv.txt"
CMT_CONV_VAR=16 timeout -k 10 200 python -u -m pytest tests/test_gpu_split.py -v -k "conv3x3_nchw" \
    --timeout 150 --timeout-method thread > "$OUT/tests_v4.log" 2>&1
rc=$?
[[ $rc -eq 0 || $rc -eq 1 ]] || { echo "v4 tests rc=$rc"; tail -30 "$OUT/tests_v4.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests_v4.log" | tail -2
for v in 16 0 16 0 20; do
    echo -n "conv var $v: " >> "$OUT/conv.txt"
    CMT_CONV_VAR=$v timeout -k 10 120 python -u dev/kernel_probe.py convh --time 2>/dev/null >> "$OUT/conv.txt" \
        || { echo "conv probe failed"; tail -5 "$OUT/conv.txt"; exit 1; }
done
grep "conv var" "$OUT/conv.txt"
for v in 1 0 1 0; do
    env CMT_ATTN_US=$v CMT_ATTN_VARIANT=us$v timeout -k 10 120 python -u dev/attn_exp.py --dtype f16 --nk 56400 --bound \
        --round --qs >> "$OUT/attn.txt" 2>/dev/null || { echo "attn_exp failed"; tail -5 "$OUT/attn.txt"; exit 1; }
done
grep attn "$OUT/attn.txt"
CMT_ATTN_US=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py -v -rA --timeout 200 \
    --timeout-method thread > "$OUT/fullsize_us.log" 2>&1
rc=$?
[[ $rc -eq 0 || $rc -eq 1 ]] || { echo "fullsize rc=$rc"; tail -30 "$OUT/fullsize_us.log"; exit 1; }
grep -E "passed|failed" "$OUT/fullsize_us.log" | tail -2
mkdir -p "$OUT/trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref --no-recompute --no-traffic \
    > "$OUT/trace/bench.json" 2> "$OUT/trace/trace.log" || { echo "trace failed"; tail -20 "$OUT/trace/trace.log"; exit 1; }
cat "$OUT/trace/bench.json"
