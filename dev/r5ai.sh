#!/bin/bash
# Round-5 step ai: the training decoder's forward / backward as HIP graphs (OPTIONS.train_graph) with
# the attention dropout seed read on the device (ABI 22): training tests, then the coop training
# bench graph on / off and the host profile.
set -uo pipefail
TAG=${1:-r5ai}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_head.py tests/test_gpu_train_kernels.py tests/test_gpu_0_dp_train.py \
    -m gpu -v -x --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error|error|assert" "$OUT/tests.log" | head -30; exit 1; }
grep -E "HIP graphs" "$OUT/tests.log" | head -3
for i in 1 2; do
    for g in 1 0; do
        CMT_TRAIN_GRAPH=$g timeout -k 10 300 python -u bench.py --train --workload coop --steps 30 --warmup 5 \
            > "$OUT/train_${g}_$i.json" 2> "$OUT/train_${g}_$i.log" || { echo "train $g failed"; tail -20 "$OUT/train_${g}_$i.log"; exit 1; }
        echo "graph=$g $(python -c "import json; d=json.load(open('$OUT/train_${g}_$i.json')); print(d['value'], 'steps/s', d['ms_per_step'], 'ms')")"
    done
done
timeout -k 10 400 python -u dev/train_host_profile.py > "$OUT/host.txt" 2> "$OUT/host.log" || { tail "$OUT/host.log"; exit 1; }
grep "issue" "$OUT/host.txt"
