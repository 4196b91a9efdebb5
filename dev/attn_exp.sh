#!/bin/bash
# Run attn_exp.py for a list of "TAG:ENV=VAL,ENV=VAL" variants (one process each)
# at the fusion and lidar cross-attention shapes.
#   gpurun -- bash dev/attn_exp.sh OUT "base:" "pp0:CMT_ATTN_PP=0" ...
set -uo pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for spec in "$@"; do
    tag=${spec%%:*}; envs=${spec#*:}
    for nk in 56400 32400; do
        ( export CMT_ATTN_VARIANT=$tag; IFS=','; for e in $envs; do [[ -n $e ]] && export "$e"; done; unset IFS
          timeout -k 5 90 python3 dev/attn_exp.py --nk $nk --bound --check ${EXTRA:-} ) \
          >> "$OUT/attn_exp.txt" 2>&1
        rc=$?
        if [[ $rc -ne 0 ]]; then echo "variant $tag nk $nk failed rc=$rc"; tail -5 "$OUT/attn_exp.txt"; exit $rc; fi
    done
done
cat "$OUT/attn_exp.txt"
