#!/bin/bash
# Round-4 step r: long-key fp16 training attention (core forward with the row statistic, LDS-resident
# dK/dV, K/V-streaming dQ): kernel tests vs float64 autograd, head training tests, training bench + table.
set -uo pipefail
TAG=${1:-r4w}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_kernels.py -v -k "attention or layernorm" --timeout 200 \
    --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "tests rc=$rc"; tail -30 "$OUT/tests.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests.log" | tail -1
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_head.py -v --timeout 200 --timeout-method thread \
    > "$OUT/tests_head.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "head tests rc=$rc"; tail -30 "$OUT/tests_head.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests_head.log" | tail -1
for v in 1; do
    CMT_TRAIN_ATTN_FAST=$v timeout -k 10 300 python -u bench.py --train --workload coop --steps 30 --warmup 5 \
        > "$OUT/train_$v.json" 2> "$OUT/train_$v.log" || { echo "train bench failed"; tail -5 "$OUT/train_$v.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/train_$v.json'));print('fast$v', d['value'], d['ms_per_step'])" | tee -a "$OUT/train.txt"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/train_trace" -o run --output-format csv -- \
    python3 bench.py --train --workload coop --steps 20 --warmup 3 > "$OUT/train_trace.json" 2> "$OUT/train_trace.log" || { echo "trace failed"; exit 1; }
python3 dev/trace_table.py "$OUT/train_trace" 23 > "$OUT/train_table.txt"
head -24 "$OUT/train_table.txt" | cut -c1-160
cp "$OUT"/train_trace/*kernel_stats.csv "$OUT/train_kernel_stats.csv" 2>/dev/null
rm -rf "$OUT/train_trace"
echo done
