#!/bin/bash
# SQ counters of the f16 'ref' cross-attention launch, software-pipelined (CMT_ATTN_SP=1)
# vs ping-pong (CMT_ATTN_SP=0), and HIP-event timings.
#   gpurun --timeout 600 -- bash dev/r4_pmc.sh TAG
set -uo pipefail
TAG=${1:-r4e}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for m in 1 0; do
    CMT_ATTN_SP=$m bash dev/attn_pmc.sh "$TAG/sp$m" --dtype f16 --nk 56400 --bound --round > "$OUT/pmc_sp$m.txt" 2>&1 \
        || { echo "pmc $m failed"; tail -20 "$OUT/pmc_sp$m.txt"; exit 1; }
done
for v in 1 0 5 1 0 5; do
    env CMT_ATTN_SP=$v CMT_ATTN_VARIANT=sp$v timeout -k 10 120 python -u dev/attn_exp.py --dtype f16 --nk 56400 --bound \
        --round --qs >> "$OUT/attn.txt" 2>&1 || { echo "attn_exp failed"; tail -20 "$OUT/attn.txt"; exit 1; }
done
grep attn "$OUT/attn.txt"
grep -h "derived\|mean_duration\|SQ_\|GRBM" "$OUT"/sp1/pass*/*/*_summary.json "$OUT"/sp1/pass*/*_summary.json 2>/dev/null | head -5
