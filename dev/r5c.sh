#!/bin/bash
# Round-5 step c: the attention-mix issue probe with LDS fragment reads and barriers at 2-4
# waves/SIMD; the new GPU tests (graph-path range guard, all-layer golden logits, full-size
# configs[4] parity); the default bench line twice (range-guard cost).
set -uo pipefail
TAG=${1:-r5c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 180 ./dev/issue_probe > "$OUT/issue_probe.txt" 2>&1 || { echo "probe failed"; cat "$OUT/issue_probe.txt"; exit 1; }
cat "$OUT/issue_probe.txt"
timeout -k 10 500 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_head.py tests/test_golden.py tests/test_gpu_stress4.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -12 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error" "$OUT/tests.log" | head -20; exit 1; }
timeout -k 10 60 python dev/kernel_probe.py kv --time | grep "per launch"
for i in 1 2; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.log" \
        || { echo "bench failed"; tail -20 "$OUT/bench_$i.log"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_$i.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms', 'attn', d['roofline']['avg_launch_ms'], d['roofline']['frac'], 'bf16', d.get('bf16_policy'))"
done
