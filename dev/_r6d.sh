set -uo pipefail
OUT=gpurun_out/r6d; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_head.py -q --timeout 300 --timeout-method thread -k "outlier or fullsize" > $OUT/tests.log 2>&1
grep -E "passed|failed" $OUT/tests.log | tail -2; grep -E "^training step|two-agent|full-size" $OUT/tests.log | cut -c1-1200
timeout -k 10 300 python3 -u dev/train_host_profile.py > $OUT/host_profile.txt 2>&1 || { echo "host profile failed"; tail $OUT/host_profile.txt; }
head -3 $OUT/host_profile.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --train --workload coop --steps 20 --warmup 5 > $OUT/train.json 2> $OUT/trace.log || { echo "trace failed"; tail $OUT/trace.log; exit 1; }
cat $OUT/train.json
python3 dev/trace_table.py $OUT/trace 25 70 > $OUT/train_kernel_table.txt 2>&1; head -75 $OUT/train_kernel_table.txt | cut -c1-200
find $OUT/trace -name "*.db" -delete
