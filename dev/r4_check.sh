#!/bin/bash
# Round-4 check: attention + chain tests, head path tests, full-size parity, smoke, a short bench.
set -uo pipefail
TAG=${1:-r4h}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_head.py -v -k "${K:-f16_long or pipelined or path_selections or chain or fusion or lidar}" \
    --timeout 150 --timeout-method thread -rA > "$OUT/tests.log" 2>&1
rc=$?
# rc 1: assertion failures (keep measuring); anything else (crash, timeout): stop here
[[ $rc -eq 0 || $rc -eq 1 ]] || { echo "tests rc=$rc"; tail -30 "$OUT/tests.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests.log" | tail -2
for v in 1 0; do
    env CMT_ATTN_SP=$v CMT_ATTN_VARIANT=sp$v timeout -k 10 120 python -u dev/attn_exp.py --dtype f16 --nk 56400 --bound \
        --round --qs >> "$OUT/attn.txt" 2>&1 || { echo "attn_exp failed"; tail -20 "$OUT/attn.txt"; exit 1; }
done
grep attn "$OUT/attn.txt"
for v in ${KV_VARIANTS:-0 1 2 3 5 9 13 0 1 3}; do
    echo -n "kv sched $v: " >> "$OUT/kv.txt"
    CMT_KV_SCHED=$v timeout -k 10 120 python -u dev/kernel_probe.py kv --time 2>/dev/null >> "$OUT/kv.txt" || { echo "kv probe failed"; tail -5 "$OUT/kv.txt"; exit 1; }
done
grep "kv sched" -A1 "$OUT/kv.txt"
for v in ${CONV_VARIANTS:-0 1 2 4 8 12 0 1 2}; do
    echo -n "conv var $v: " >> "$OUT/conv.txt"
    CMT_CONV_VAR=$v timeout -k 10 120 python -u dev/kernel_probe.py convh --time >> "$OUT/conv.txt" 2>&1 || { echo "conv probe failed"; tail -5 "$OUT/conv.txt"; exit 1; }
done
grep "conv var" -A1 "$OUT/conv.txt"
for c in 1 0; do
    CMT_CHAIN=$c timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-ref --no-traffic \
        --no-recompute > "$OUT/bench_chain$c.json" 2> "$OUT/bench_chain$c.log" || { echo "bench failed"; tail -20 "$OUT/bench_chain$c.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_chain$c.json'));print('chain $c', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
