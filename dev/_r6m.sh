set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mlp.py "tests/test_gpu_head.py::test_rv_rows_one_launch_bit_exact" tests/test_gpu_train_kernels.py 2>&1 | tail -2 || exit 1
timeout -k 10 120 env TAG=new python3 dev/mlp_geo_probe.py || exit 1
NOSIDE="--no-cpu-baseline --no-traffic --no-ref --no-side --no-recompute"
for i in 1 2; do timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 $NOSIDE > gpurun_out/r6m_b$i.json 2>/dev/null || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r6m_b$i.json'));print('bench',d['value'],d['roofline']['frac'])"; done
for i in 1 2; do timeout -k 10 200 python3 bench.py --train --workload coop --steps 30 --warmup 5 > gpurun_out/r6m_t$i.json 2>/dev/null || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r6m_t$i.json'));print('train',d['value'])"; done
