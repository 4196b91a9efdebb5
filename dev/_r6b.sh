set -uo pipefail
OUT=gpurun_out/r6b; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OLD=$GRAFT_REPO_ROOT/cmt-cooperative-perception_amd/lib/exp/libcmt_hip_convold.so
NEW=$GRAFT_REPO_ROOT/cmt-cooperative-perception_amd/lib/libcmt_hip.so
timeout -k 10 120 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 100 -k "conv3x3_nchw" 2>&1 | tail -2
for i in 1 2 3; do
  CMT_HIP_LIB=$NEW timeout -k 10 60 python3 dev/kernel_probe.py convh --time 2>&1 | grep us | sed 's/^/new /'
  CMT_HIP_LIB=$OLD timeout -k 10 60 python3 dev/kernel_probe.py convh --time 2>&1 | grep us | sed 's/^/old /'
done
for v in new old; do
  L=$NEW; [[ $v == old ]] && L=$OLD
  CMT_HIP_LIB=$L timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/pmc_$v -o run --output-format csv -- python3 dev/kernel_probe.py convh --iters 3 > $OUT/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $OUT/pmc_$v.log; exit 1; }
  f=$(find $OUT/pmc_$v -name "*counter_collection.csv" | head -1); python3 - "$f" $v <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "conv_halo" in r.get("Kernel_Name", ""):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: sum(v) / len(v) for k, v in acc.items()}, "launches", {k: len(v) for k, v in acc.items()})
PY
done
for nq in 900 768 1024 640; do
  timeout -k 10 60 python3 dev/attn_exp.py --dtype fp16 --qs --round --bound --nk 56400 --nq $nq --splits 8 2>&1 | grep attn
done
for s in 6 7 9 10; do
  timeout -k 10 60 python3 dev/attn_exp.py --dtype fp16 --qs --round --bound --nk 56400 --nq 768 --splits $s 2>&1 | grep attn
done
