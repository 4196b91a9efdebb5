#!/bin/bash
# Round-4 probe: cross-attention core timings (QS vs fold) + full-size parity sweep.
#   gpurun --timeout 900 -- bash dev/r4_probe.sh TAG
set -uo pipefail
TAG=${1:-r4a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [[ -x dev/coexec_probe ]]; then
    timeout -k 10 120 ./dev/coexec_probe > "$OUT/coexec.txt" 2>&1 || { echo "coexec failed"; cat "$OUT/coexec.txt"; exit 1; }
    cat "$OUT/coexec.txt"
fi
for v in "--qs" ""; do
    timeout -k 10 120 python -u dev/attn_exp.py --dtype f16 --nk 56400 --bound --round --check $v >> "$OUT/attn.txt" 2>&1 \
        || { echo "attn_exp failed"; tail -20 "$OUT/attn.txt"; exit 1; }
done
cat "$OUT/attn.txt"
timeout -k 10 700 python -u tests/diag/parity_sweep.py ${SWEEP_ARGS:-} --out "$OUT/parity_sweep.json" > "$OUT/parity_sweep.txt" 2>&1 \
    || { echo "sweep failed"; tail -30 "$OUT/parity_sweep.txt"; exit 1; }
cat "$OUT/parity_sweep.txt"
