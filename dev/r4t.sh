#!/bin/bash
# Round-4 step t: cmt_mlp2_x3 LDS fragment prefetch distance 2 / 3 / 4 (tests + timing)
set -uo pipefail
TAG=${1:-r4t}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for pd in 2 3 4 2 3 4; do
    CMT_MLP_PD=$pd timeout -k 10 200 python -u -m pytest tests/test_gpu_mlp.py -q --timeout 150 --timeout-method thread \
        > "$OUT/tests_$pd.log" 2>&1 || { echo "tests pd=$pd failed"; tail -20 "$OUT/tests_$pd.log"; exit 1; }
    echo -n "pd=$pd $(grep -E 'passed|failed' "$OUT/tests_$pd.log" | tail -1) " | tee -a "$OUT/mlp.txt"
    CMT_MLP_PD=$pd timeout -k 10 120 python -u dev/mlp_probe.py 2>/dev/null | grep "M=24000" | tee -a "$OUT/mlp.txt"
done
