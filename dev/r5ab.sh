#!/bin/bash
# Round-5 step ab: the training shared_conv weight gradient's split-K (2 vs 4 / 8 / 16).
set -uo pipefail
TAG=${1:-r5ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMT_DW_KSPLIT=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_train_head.py -m gpu -q -x -k "grads_match" --timeout 200 \
    --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?; tail -1 "$OUT/tests.log"; [[ $rc -eq 0 ]] || exit 1
for v in 2 8 16 4 2 8; do
    CMT_DW_KSPLIT=$v timeout -k 10 300 python3 -u bench.py --train --workload coop --steps 30 --warmup 5 > "$OUT/train_$v.json" 2> "$OUT/train_$v.log" \
        || { echo "train $v failed"; tail "$OUT/train_$v.log"; exit 1; }
    echo "ksplit $v $(python -c "import json; d=json.load(open('$OUT/train_$v.json')); print(d['value'], 'steps/s', d['ms_per_step'], 'ms')")"
done
