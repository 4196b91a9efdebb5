#!/bin/bash
# Round-5 step ad: the training bf16x3 GEMM (first run: X3_DEPTH k-steps of loads in flight, rejected)
# -- then the transposed [k][row] image (r5ae/af), 128 x 128 tiles (r5an, nobig), then the k-wave split of small products (r5ap: base vs nokw)
# tests, and the coop training bench A/B.
set -uo pipefail
TAG=${1:-r5ad}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base nokw; do
    lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v != base ]] && lib=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_$v.so
    CMT_HIP_LIB=$lib timeout -k 10 120 python dev/gemm_probe.py 2>&1 | sed "s/^/$v /" || { echo "probe $v failed"; exit 1; }
done
timeout -k 10 600 python -u -m pytest tests/test_host.py tests/test_gpu_train_kernels.py tests/test_gpu_train_head.py -m gpu -q -x --timeout 300 \
    --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit 1; }
for i in 1 2 3; do
    for v in base nokw; do
        lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v != base ]] && lib=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_$v.so
        CMT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --train --workload coop --steps 30 --warmup 5 \
            > "$OUT/train_${v}_$i.json" 2> "$OUT/train_${v}_$i.log" || { echo "train $v failed"; tail -5 "$OUT/train_${v}_$i.log"; exit 1; }
        echo "$v $(python -c "import json; d=json.load(open('$OUT/train_${v}_$i.json')); print(d['value'], 'steps/s', d['ms_per_step'], 'ms')")"
    done
done
