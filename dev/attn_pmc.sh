#!/bin/bash
# SQ counter passes over the cross-attention probe (dev/attn_probe.py), one
# rocprofv3 --pmc run per counter group (8 SQ slots max per pass), plus the
# counter list of this box.  Output: gpurun_out/TAG/{counters.txt,pass*/}.
#   gpurun --timeout 600 -- bash dev/attn_pmc.sh TAG [probe args]
set -uo pipefail
TAG=${1:-pmc}
shift || true
OUT=gpurun_out/${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || echo "counter list failed"
PROBE="dev/attn_probe.py --iters 5 ${*:---fold}"
i=0
for group in \
    "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
    "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" \
    "SQ_INST_CYCLES_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM"; do
    i=$((i + 1))
    rc=0
    timeout -s KILL 60 rocprofv3 --pmc $group -d "$OUT/pass$i" -o run -- python3 $PROBE > "$OUT/pass$i.log" 2>&1 || rc=$?
    echo "pass $i rc=$rc: $group"
    if [[ $rc -ne 0 ]]; then tail -5 "$OUT/pass$i.log"; fi
    if [[ $rc -eq 134 || $rc -eq 139 ]]; then exit $rc; fi
done
for db in "$OUT"/pass*/*/*.db "$OUT"/pass*/*.db; do
    [[ -f $db ]] && python3 dev/pmc_summary.py "$db" --match attn \
        > "${db%.db}_summary.json" && cat "${db%.db}_summary.json"
done
# keep what gpurun copies back small: the summaries stay, the databases go
find "$OUT" -name "*.db" -delete
exit 0
