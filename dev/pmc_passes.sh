#!/bin/bash
# Counter passes, one rocprofv3 --pmc run per group (gfx950 slot limits: <= 8 SQ,
# FETCH_SIZE and WRITE_SIZE in passes of their own), over one probe command.
#   bash dev/pmc_passes.sh OUTDIR MATCH probe.py args...
set -uo pipefail
OUT=$1; MATCH=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for group in \
    "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
    "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" \
    "SQ_INST_CYCLES_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM" \
    "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    rc=0
    timeout -s KILL 90 rocprofv3 --pmc $group -d "$OUT/pass$i" -o run -- python3 "$@" > "$OUT/pass$i.log" 2>&1 || rc=$?
    echo "pass $i rc=$rc: $group"
    if [[ $rc -ne 0 ]]; then tail -5 "$OUT/pass$i.log"; exit $rc; fi
done
python3 - "$OUT" "$MATCH" <<'PY'
import glob, json, sys
sys.path.insert(0, "dev")
from pmc_summary import summarise
out, match = sys.argv[1], sys.argv[2]
merged = {}
for db in sorted(glob.glob(f"{out}/pass*/**/*.db", recursive=True)):
    for k, v in summarise(db, match).items():
        merged.setdefault(k, {}).update(v)
json.dump(merged, open(f"{out}/summary.json", "w"), indent=1)
print(json.dumps(merged, indent=1))
PY
find "$OUT" -name "*.db" -delete
exit 0
