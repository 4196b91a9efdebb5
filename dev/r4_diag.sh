#!/bin/bash
set -uo pipefail
OUT=gpurun_out/${1:-r4d}
mkdir -p "$OUT"
for m in 1 3; do
    CMT_ATTN_SP=$m timeout -k 10 180 python -u dev/sp_diag.py > "$OUT/diag_$m.txt" 2>&1 || { cat "$OUT/diag_$m.txt"; exit 1; }
    echo "== mode $m"; cat "$OUT/diag_$m.txt"
done
