#!/bin/bash
# Round-5 step d: the persistent kvproj (product lib) and the tile-at-a-time attention kernel
# (dev lib lib/exp/libcmt_hip_tt.so, CMT_ATTN_EXP=4): attention / kvproj parity tests on both,
# the golden per-key log, attention microbenchmark and bench A/B.
set -uo pipefail
TAG=${1:-r5d}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
TT=cmt-cooperative-perception_amd/lib/exp/libcmt_hip_tt.so
true || timeout -k 10 300 python -u -m pytest tests/test_golden.py -m gpu -q \
    --timeout 200 --timeout-method thread > "$OUT/tests_base.log" 2>&1
tail -8 "$OUT/tests_base.log"
CMT_HIP_LIB=$TT timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_kernels.py -m gpu -x -q \
    -k "attention or attn" --timeout 200 --timeout-method thread > "$OUT/tests_tt.log" 2>&1
rc=$?; tail -3 "$OUT/tests_tt.log"; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error" "$OUT/tests_tt.log" | head -20; exit 1; }
timeout -k 10 60 python dev/kernel_probe.py kv --time | grep "per launch"
for v in base tt base tt; do
    lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v == tt ]] && lib=$TT
    CMT_HIP_LIB=$lib timeout -k 10 120 python -u dev/attn_exp.py --dtype f16 --nk 56400 --bound --qs --round --check --tag $v \
        >> "$OUT/attn.txt" 2>&1 || { echo "attn_exp $v failed"; tail -20 "$OUT/attn.txt"; exit 1; }
done
grep attn "$OUT/attn.txt"
for v in base tt base tt; do
    lib=cmt-cooperative-perception_amd/lib/libcmt_hip.so; [[ $v == tt ]] && lib=$TT
    CMT_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ref --no-traffic --no-recompute --steps 40 \
        > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench $v failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    echo "$v $(python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms', 'attn', d['roofline']['avg_launch_ms'], 'ms', d['roofline']['frac'])")"
done
