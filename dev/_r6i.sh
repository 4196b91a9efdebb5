set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=cmt-cooperative-perception_amd/lib
timeout -k 10 120 env TAG=base python3 dev/mlp_geo_probe.py || exit 1
for d in 8 24 3 7 31; do
  timeout -k 10 120 env TAG=d$d CMT_HIP_LIB=$PWD/$L/exp/libcmt_hip_d$d.so python3 dev/mlp_geo_probe.py || exit 1
done
timeout -k 10 120 env TAG=base python3 dev/mlp_geo_probe.py || exit 1
