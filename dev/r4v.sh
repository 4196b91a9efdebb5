#!/bin/bash
# Round-4 step v: the dQ kernel with 64 queries per wave (CMT_TRAIN_DQ_QB=2, default) vs 32:
# long-key training attention tests for both, training A/B, kernel table.
set -uo pipefail
TAG=${1:-r4v}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 2 1; do
    CMT_TRAIN_DQ_QB=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_train_kernels.py -q -k "attention" \
        --timeout 200 --timeout-method thread > "$OUT/tests_$v.log" 2>&1
    rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "tests rc=$rc"; tail -30 "$OUT/tests_$v.log"; exit 1; }
    echo "qb$v $(grep -E 'passed|failed' "$OUT/tests_$v.log" | tail -1)"
done
for v in 2 1 2 1; do
    CMT_TRAIN_DQ_QB=$v timeout -k 10 300 python -u bench.py --train --workload coop --steps 30 --warmup 5 \
        > "$OUT/train_$v.json" 2> "$OUT/train_$v.log" || { echo "train bench failed"; tail -5 "$OUT/train_$v.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/train_$v.json'));print('qb$v', d['value'], d['ms_per_step'])" | tee -a "$OUT/train.txt"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/train_trace" -o run --output-format csv -- \
    python3 bench.py --train --workload coop --steps 20 --warmup 3 > "$OUT/train_trace.json" 2> "$OUT/train_trace.log" || { echo "trace failed"; exit 1; }
python3 dev/trace_table.py "$OUT/train_trace" 23 > "$OUT/train_table.txt"
grep -E "dq2|dkv2|attn_pb2" "$OUT/train_table.txt" | cut -c1-150
cp "$OUT"/train_trace/*kernel_stats.csv "$OUT/train_kernel_stats.csv" 2>/dev/null
rm -rf "$OUT/train_trace"
echo done
