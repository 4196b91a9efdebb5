set -uo pipefail
OUT=gpurun_out/r6e; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_train_head.py tests/test_gpu_train_kernels.py tests/test_gpu_0_dp_train.py tests/test_gpu_cli.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/tests.log | tail -2; grep -E "in place|FAILED|Error" $OUT/tests.log | head -20 | cut -c1-600
[[ $rc -eq 0 ]] || exit 1
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --train --workload coop --steps 30 --warmup 5 > $OUT/train$i.json 2> $OUT/train$i.log || { echo "train failed"; tail $OUT/train$i.log; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/train$i.json')); print('train', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python3 -u dev/train_host_profile.py > $OUT/host_profile.txt 2>&1 || { echo "host profile failed"; tail $OUT/host_profile.txt; }
head -3 $OUT/host_profile.txt
