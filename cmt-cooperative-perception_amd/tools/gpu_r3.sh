set -o pipefail
mkdir -p gpurun_out/r3b
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 150 --timeout-method thread -rA > gpurun_out/r3b/split.log 2>&1; rc=$?
tail -30 gpurun_out/r3b/split.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 150 --timeout-method thread -k "attention or gemm" > gpurun_out/r3b/kern.log 2>&1; rc=$?
tail -15 gpurun_out/r3b/kern.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-batch2 > gpurun_out/r3b/bench.json 2> gpurun_out/r3b/bench.log; rc=$?
cat gpurun_out/r3b/bench.json; tail -5 gpurun_out/r3b/bench.log
exit $rc
