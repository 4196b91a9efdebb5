#!/bin/bash
# Round-5 step b: the full GPU suite on the pruned library (BatchNorm partial sums, training
# attention workspace check), then fresh counters (SQ + HBM traffic) of the four 'ref' kernels
# the verdict names: kvproj_x3, conv_halo_x3, mlp2_x3, attn_pb2 + combine.
set -uo pipefail
TAG=${1:-r5b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error|error" "$OUT/tests.log" | head -20; exit 1; }
bash dev/r5_pmc.sh "$OUT/kv" kvproj dev/kernel_probe.py kv --iters 5 > "$OUT/kv.txt" 2>&1 || { tail "$OUT/kv.txt"; exit 1; }
bash dev/r5_pmc.sh "$OUT/convh" conv_halo dev/kernel_probe.py convh --iters 5 > "$OUT/convh.txt" 2>&1 || { tail "$OUT/convh.txt"; exit 1; }
bash dev/r5_pmc.sh "$OUT/mlp" mlp2 dev/kernel_probe.py mlp --iters 5 > "$OUT/mlp.txt" 2>&1 || { tail "$OUT/mlp.txt"; exit 1; }
bash dev/r5_pmc.sh "$OUT/attn" attn dev/attn_probe.py --iters 5 --dtype f16 --nk 56400 --bound --round > "$OUT/attn.txt" 2>&1 || { tail "$OUT/attn.txt"; exit 1; }
for w in kv convh mlp; do timeout -k 10 60 python dev/kernel_probe.py $w --time | grep "per launch"; done
echo done
