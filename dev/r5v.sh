#!/bin/bash
# Round-5 step m: the camera memory rows in one launch (ABI 20):
# head tests incl. the bit-exact on/off test, full-size parity, then bench A/B.
set -uo pipefail
TAG=${1:-r5v}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_head.py tests/test_golden.py tests/test_gpu_fullsize.py tests/test_gpu_stress4.py -m gpu -q -x \
    --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit 1; }
grep -E "bit-exact|fusion|golden" "$OUT/tests.log" | head -5
for v in on off on off; do
    cc=1; [[ $v == off ]] && cc=0
    CMT_RV_GEO=$cc timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ref --no-traffic --no-recompute --steps 50 \
        > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench $v failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    echo "$v $(python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms', d['roofline']['avg_launch_ms'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic --no-ref --no-recompute > "$OUT/bench_trace.json" 2> "$OUT/trace.log" \
    || { echo "trace failed"; tail "$OUT/trace.log"; exit 1; }
python3 dev/timeline.py "$OUT/trace" 4 > "$OUT/timeline.txt" 2>&1 || true
tail -1 "$OUT/timeline.txt"
