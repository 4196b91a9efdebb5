#!/bin/bash
# Round-5 step bc: the task heads' tap gather as one autograd op and the agents' query split by split()
# (base) vs pad + slices + cat and slicing (CMT_TAPS_EXP=0): coop training bench, 4 alternating pairs.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5bc
for i in 1 2 3 4; do
    for v in 1 0; do
        CMT_TAPS_EXP=$v timeout -k 10 300 python -u bench.py --train --workload coop --steps 40 --warmup 5 \
            > gpurun_out/r5bc/b_${v}_$i.json 2> gpurun_out/r5bc/b_${v}_$i.log || { echo "train $v failed"; exit 1; }
        echo "new=$v $(python -c "import json; d=json.load(open('gpurun_out/r5bc/b_${v}_$i.json')); print(d['value'], 'steps/s')")"
    done
done
