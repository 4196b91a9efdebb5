#!/bin/bash
# Attention kernel A/B: correctness tests of the f16 long-key kernels, then
# HIP-event timings of the software-pipelined kernel vs the ping-pong kernel.
#   gpurun --timeout 600 -- bash dev/r4_attn.sh TAG [pytest -k expr]
set -uo pipefail
TAG=${1:-r4b}
K=${2:-"f16_long or pipelined or bounded"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_kernels.py -k "$K" -x -q \
    --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
for v in ${VARIANTS:-"CMT_ATTN_SP=1:--qs" "CMT_ATTN_SP=3:--qs" "CMT_ATTN_SP=5:--qs" "CMT_ATTN_SP=7:--qs" "CMT_ATTN_SP=0:--qs" "CMT_ATTN_SP=1:--qs" "CMT_ATTN_SP=3:--qs" "CMT_ATTN_SP=5:--qs" "CMT_ATTN_SP=7:--qs" "CMT_ATTN_SP=0:--qs"}; do
    e=${v%%:*}; a=${v#*:}
    env $e CMT_ATTN_VARIANT=$e timeout -k 10 120 python -u dev/attn_exp.py --dtype f16 --nk 56400 --bound --round --check $a \
        >> "$OUT/attn.txt" 2>&1 || { echo "attn_exp failed"; tail -20 "$OUT/attn.txt"; exit 1; }
done
grep attn "$OUT/attn.txt"
