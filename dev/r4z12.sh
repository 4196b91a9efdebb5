#!/bin/bash
# Round-4 step z12: query embedding + layer-0 prologue on the side stream after shared_conv (1) or beside it (0):
# head path tests, frame A/B (alternating).
set -uo pipefail
TAG=${1:-r4z12}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_head.py -v -k "path_selections or fusion or coop" \
    --timeout 150 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "tests rc=$rc"; tail -30 "$OUT/tests.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests.log" | tail -1
for v in 1 0 1 0 1 0; do
    CMT_QPOS_AFTER_CONV=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-ref --no-traffic \
        --no-recompute > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('qlate$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" | tee -a "$OUT/bench.txt"
done
echo done
