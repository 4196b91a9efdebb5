#!/bin/bash
# Round-5 step as: the agents' training decoders as one walk (query side batched over agents) vs one
# walk per agent -- then (r5at) the graph-replayed batched walk vs op by op: training tests, bench A/B, host profile.
set -uo pipefail
TAG=${1:-r5as}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_head.py tests/test_gpu_0_dp_train.py -m gpu -q -x \
    --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -1 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit 1; }
grep -E "two-agent|HIP graphs" "$OUT/tests.log" | head -4
for i in 1 2 3; do
    for v in 1 0; do
        CMT_BATCH_AGENTS_EXP=$v timeout -k 10 300 python -u bench.py --train --workload coop --steps 30 --warmup 5 \
            > "$OUT/b_${v}_$i.json" 2> "$OUT/b_${v}_$i.log" || { echo "train $v failed"; tail -5 "$OUT/b_${v}_$i.log"; exit 1; }
        echo "batched=$v $(python -c "import json; d=json.load(open('$OUT/b_${v}_$i.json')); print(d['value'], 'steps/s')")"
    done
done
timeout -k 10 400 python -u dev/train_host_profile.py > "$OUT/host.txt" 2> "$OUT/host.log" || { tail "$OUT/host.log"; exit 1; }
grep "issue" "$OUT/host.txt"
