#!/bin/bash
set -uo pipefail
OUT=gpurun_out/${1:-r4f}
mkdir -p "$OUT"
timeout -k 10 120 ./dev/slot_probe > "$OUT/slot.txt" 2>&1 || { cat "$OUT/slot.txt"; exit 1; }
cat "$OUT/slot.txt"
for v in 1 17 0 1 17 0; do
    env CMT_ATTN_SP=$v CMT_ATTN_VARIANT=sp$v timeout -k 10 120 python -u dev/attn_exp.py --dtype f16 --nk 56400 --bound \
        --round --qs >> "$OUT/attn.txt" 2>&1 || { echo "attn_exp failed"; tail -20 "$OUT/attn.txt"; exit 1; }
done
grep attn "$OUT/attn.txt"
