#!/bin/bash
# Round-5 step j: frame start with the camera upload + frustum coordinates on the second stream
# (CMT_FORK_FIRST=1: the conv is the frame's first main-stream kernel) vs the committed order.
set -uo pipefail
TAG=${1:-r5j}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMT_FORK_FIRST=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_fullsize.py -m gpu -q -x \
    --timeout 200 --timeout-method thread > "$OUT/tests_ff.log" 2>&1
rc=$?; tail -3 "$OUT/tests_ff.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error" "$OUT/tests_ff.log" | head; exit 1; }
for v in ff base ff base; do
    ff=0; [[ $v == ff ]] && ff=1
    CMT_FORK_FIRST=$ff timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ref --no-traffic --no-recompute --steps 50 \
        > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench $v failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    echo "$v $(python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms')")"
done
CMT_FORK_FIRST=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic --no-ref --no-recompute > "$OUT/bench_trace.json" 2> "$OUT/trace.log" \
    || { echo "trace failed"; tail "$OUT/trace.log"; exit 1; }
python3 dev/timeline.py "$OUT/trace" 4 > "$OUT/timeline_ff.txt" 2>&1 || true
tail -1 "$OUT/timeline_ff.txt"
