set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$PWD/cmt-cooperative-perception_amd/lib/exp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mlp.py "tests/test_gpu_head.py::test_rv_rows_one_launch_bit_exact" 2>&1 | tail -3 || exit 1
for v in base v0 v1 v2 base v0; do
  if [[ $v == base ]]; then timeout -k 10 120 env TAG=$v python3 dev/mlp_geo_probe.py || exit 1
  else timeout -k 10 120 env TAG=$v CMT_HIP_LIB=$L/libcmt_hip_$v.so python3 dev/mlp_geo_probe.py || exit 1; fi
done
