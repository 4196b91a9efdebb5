#!/bin/bash
# Round-5 step am: the camera-matrix upload on the second stream (the conv the frame's first node)
# vs on the main stream ahead of the conv: head tests, bench A/B, one timeline.
set -uo pipefail
TAG=${1:-r5am}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_head.py tests/test_golden.py -m gpu -q -x \
    --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -1 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit 1; }
for i in 1 2 3; do
    for v in 1 0; do
        CMT_LATE_CAMS_EXP=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ref --no-traffic --no-recompute --steps 100 \
            > "$OUT/bench_${v}_$i.json" 2> "$OUT/bench_${v}_$i.log" || { echo "bench $v failed"; tail -20 "$OUT/bench_${v}_$i.log"; exit 1; }
        echo "late_cams=$v $(python -c "import json; d=json.load(open('$OUT/bench_${v}_$i.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms')")"
    done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic --no-ref --no-recompute > "$OUT/bench_trace.json" 2> "$OUT/trace.log" \
    || { echo "trace failed"; tail "$OUT/trace.log"; exit 1; }
python3 dev/timeline.py "$OUT/trace" 4 > "$OUT/timeline.txt" 2>&1 || true
head -6 "$OUT/timeline.txt"; tail -4 "$OUT/timeline.txt"
find "$OUT/trace" -name "*kernel_trace.csv" -delete
