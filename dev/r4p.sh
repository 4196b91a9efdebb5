#!/bin/bash
# Round-4 step o: split chains with the prologue loads ahead of the weight ring and a 16-step ring
# (phase stamps of both rings, head path tests, full-size parity, frame A/B ring 16 vs 8).
set -uo pipefail
TAG=${1:-r4p}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_head.py -v -k "path_selections or chain or fusion" \
    --timeout 150 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "tests rc=$rc"; tail -30 "$OUT/tests.log"; exit 1; }
grep -E "passed|failed" "$OUT/tests.log" | tail -1
for r in bar nobar; do
    echo "## $r" >> "$OUT/stamps.txt"
    CMT_CHAIN_NOBAR=$([[ $r == nobar ]] && echo 1 || echo 0) CMT_HIP_LIB=cmt-cooperative-perception_amd/lib_stamps/libcmt_hip.so timeout -k 10 200 \
        python -u dev/chain_stamps.py >> "$OUT/stamps.txt" 2>&1 || { echo "stamps failed"; tail -20 "$OUT/stamps.txt"; exit 1; }
done
cat "$OUT/stamps.txt"
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -v -rA -k "fusion or coop" --timeout 200 \
    --timeout-method thread > "$OUT/fullsize.log" 2>&1
rc=$?; [[ $rc -eq 0 || $rc -eq 1 ]] || { echo "fullsize rc=$rc"; tail -30 "$OUT/fullsize.log"; exit 1; }
grep -E "passed|failed" "$OUT/fullsize.log" | tail -1
for v in 0 1 0 1; do
    CMT_CHAIN_NOBAR=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-ref --no-traffic \
        --no-recompute > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('nobar$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" | tee -a "$OUT/bench.txt"
done
echo done
