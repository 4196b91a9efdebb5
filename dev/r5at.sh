#!/bin/bash
# Round-5 step at: the batched agents' training decoder replayed as one HIP graph (CMT_TRAIN_GRAPH=1)
# vs op by op: training tests, coop training bench A/B, host profile of both.
set -uo pipefail
TAG=${1:-r5at}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_head.py tests/test_gpu_0_dp_train.py -m gpu -q -x \
    --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -1 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit 1; }
grep -E "HIP graphs" "$OUT/tests.log" | head -2
for i in 1 2 3; do
    for g in 1 0; do
        CMT_TRAIN_GRAPH=$g timeout -k 10 300 python -u bench.py --train --workload coop --steps 30 --warmup 5 \
            > "$OUT/b_${g}_$i.json" 2> "$OUT/b_${g}_$i.log" || { echo "train $g failed"; tail -5 "$OUT/b_${g}_$i.log"; exit 1; }
        echo "graph=$g $(python -c "import json; d=json.load(open('$OUT/b_${g}_$i.json')); print(d['value'], 'steps/s')")"
    done
done
for g in 1 0; do
    CMT_TRAIN_GRAPH=$g timeout -k 10 400 python -u dev/train_host_profile.py > "$OUT/host$g.txt" 2> "$OUT/host$g.log" || { tail "$OUT/host$g.log"; exit 1; }
    echo "graph=$g $(grep issue "$OUT/host$g.txt")"
done
