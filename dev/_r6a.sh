set -uo pipefail
OUT=gpurun_out/r6a; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_kernels.py tests/test_gpu_train_head.py -x -q --timeout 200 --timeout-method thread -k "linear_bwd or range_guard or eval_after or fullsize or outlier or graph or grads_match" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [[ $rc -eq 0 ]] || { grep -E "^FAILED|Error|assert" $OUT/tests.log | head -30; exit 1; }
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.log || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
cat $OUT/bench.json
