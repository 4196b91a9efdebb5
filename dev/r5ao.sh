#!/bin/bash
# Round-5 step ao: the training GEMM's final tile rule -- training kernel / head tests, the probe,
# the coop training bench (committed line) and its kernel table.
set -uo pipefail
TAG=${1:-r5ao}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_kernels.py tests/test_gpu_train_head.py tests/test_gpu_0_dp_train.py \
    -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -1 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit 1; }
timeout -k 10 120 python dev/gemm_probe.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python3 -u bench.py --train --workload coop > "$OUT/train_coop.json" 2> "$OUT/train_coop.log" \
    || { echo "train bench failed"; tail "$OUT/train_coop.log"; exit 1; }
cat "$OUT/train_coop.json"
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --train --workload coop --steps 10 --warmup 3 > "$OUT/train_trace.json" 2> "$OUT/train_trace.log" \
    || { echo "trace failed"; tail "$OUT/train_trace.log"; exit 1; }
python3 dev/trace_table.py "$OUT/trace" 13 > "$OUT/table.txt" 2>&1 || true
head -12 "$OUT/table.txt" | cut -c1-150
find "$OUT/trace" -name "*kernel_trace.csv" -delete
