#!/bin/bash
# Round-5 step a: issue-ceiling probe of the d_h = 32 attention mix at 1-4 waves/SIMD, then the
# segment-priority variants of attn_pb2_kernel (dev libraries lib/exp/libcmt_hip_p*.so):
# attention microbenchmark at the 'ref' numerics and the default bench per library.
set -uo pipefail
TAG=${1:-r5a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
LIBD=cmt-cooperative-perception_amd/lib
timeout -k 10 120 ./dev/issue_probe > "$OUT/issue_probe.txt" 2>&1 || { echo "probe failed"; cat "$OUT/issue_probe.txt"; exit 1; }
cat "$OUT/issue_probe.txt"
for v in base p1 p2 p3; do
    lib=$LIBD/libcmt_hip.so; [[ $v != base ]] && lib=$LIBD/exp/libcmt_hip_$v.so
    CMT_HIP_LIB=$lib timeout -k 10 120 python -u dev/attn_exp.py --dtype f16 --nk 56400 --bound --qs --round --check --tag $v \
        >> "$OUT/attn.txt" 2>&1 || { echo "attn_exp $v failed"; tail -20 "$OUT/attn.txt"; exit 1; }
done
cat "$OUT/attn.txt" | grep attn
for v in base p1 p2 p3 base p1; do
    lib=$LIBD/libcmt_hip.so; [[ $v != base ]] && lib=$LIBD/exp/libcmt_hip_$v.so
    CMT_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ref --no-traffic --no-recompute --steps 40 \
        > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { echo "bench $v failed"; tail -20 "$OUT/bench_$v.log"; exit 1; }
    echo "$v $(python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print(d['value'], 'fps', d['ms_per_step'], 'ms', 'attn', d['roofline']['avg_launch_ms'], 'ms', d['roofline']['frac'])")"
done
