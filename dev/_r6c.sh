set -uo pipefail
OUT=gpurun_out/r6c; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_head.py -q --timeout 300 --timeout-method thread -k "outlier or fullsize" > $OUT/tests.log 2>&1
grep -E "passed|failed" $OUT/tests.log | tail -2; grep -E "^training step|two-agent|full-size" $OUT/tests.log | cut -c1-900
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.log || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
cat $OUT/bench.json
