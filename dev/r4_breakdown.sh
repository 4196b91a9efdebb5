#!/bin/bash
# Where the 'ref' policy's logit error comes from: split vs exact-f32 GEMMs x bounded vs
# online cross-attention offsets (fusion, full size), and exact-f32 GEMMs for one seed of
# every config (parity_sweep variant 'exact').
set -uo pipefail
OUT=gpurun_out/${1:-r4g}
mkdir -p "$OUT"
timeout -k 10 300 python -u tests/diag/ref_error_diag.py > "$OUT/ref_error_diag.txt" 2>&1 || { tail -20 "$OUT/ref_error_diag.txt"; exit 1; }
cat "$OUT/ref_error_diag.txt"
timeout -k 10 400 python -u tests/diag/parity_sweep.py --seeds 0 --variants ref exact --no-fp32-gap \
    --out "$OUT/parity_exact.json" > "$OUT/parity_exact.txt" 2>&1 || { tail -20 "$OUT/parity_exact.txt"; exit 1; }
cat "$OUT/parity_exact.txt"
