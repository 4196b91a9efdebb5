#!/bin/bash
# Round-5 step aq: the k-wave split of small training GEMMs (base) vs none (nokw): training tests,
# then kernel durations of the training step (rocprofv3) for both builds.
set -uo pipefail
TAG=${1:-r5aq}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_kernels.py tests/test_gpu_train_head.py -m gpu -q -x \
    --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -1 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit 1; }
for v in base nokw; do
    lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v != base ]] && lib=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_$v.so
    CMT_HIP_LIB=$lib timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/trace_$v" -o run --output-format csv -- \
        python3 bench.py --train --workload coop --steps 10 --warmup 3 > "$OUT/train_$v.json" 2> "$OUT/train_$v.log" \
        || { echo "trace failed"; tail "$OUT/train_$v.log"; exit 1; }
    python3 dev/trace_table.py "$OUT/trace_$v" 13 > "$OUT/table_$v.txt" 2>&1 || true
    echo "== $v: $(python3 -c "
import re
tot=0.0; g=0.0
for l in open('$OUT/table_$v.txt'):
    m=re.search(r'([0-9.]+)us/frame', l)
    if m:
        tot+=float(m.group(1))
        if 'gemm_ex3' in l: g+=float(m.group(1))
print(f'kernel time {tot/1e3:.2f} ms/step, gemm_ex3 {g/1e3:.2f} ms/step')")"
    grep gemm_ex3 "$OUT/table_$v.txt" | head -8 | cut -c1-140
    find "$OUT/trace_$v" -name "*kernel_trace.csv" -delete
done
for i in 1 2; do
    for v in base nokw; do
        lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v != base ]] && lib=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_$v.so
        CMT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --train --workload coop --steps 30 --warmup 5 \
            > "$OUT/b_${v}_$i.json" 2> "$OUT/b_${v}_$i.log" || { echo "train $v failed"; exit 1; }
        echo "$v $(python -c "import json; d=json.load(open('$OUT/b_${v}_$i.json')); print(d['value'], 'steps/s')")"
    done
done
