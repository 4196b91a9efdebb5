set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
E=$GRAFT_REPO_ROOT/cmt-cooperative-perception_amd/lib/exp
D=$GRAFT_REPO_ROOT/cmt-cooperative-perception_amd/lib/libcmt_hip.so
for L in $E/libcmt_hip_atold.so $D $E/libcmt_hip_at1.so $E/libcmt_hip_at2.so $E/libcmt_hip_at4.so $E/libcmt_hip_at7.so $E/libcmt_hip_at8.so $E/libcmt_hip_at9.so $D; do
  CMT_HIP_LIB=$L timeout -k 10 60 python3 dev/attn_train_probe.py > /tmp/p.log 2>&1 || { tail -5 /tmp/p.log; exit 1; }
  grep attn_train /tmp/p.log
done
timeout -k 10 60 python3 dev/attn_train_probe.py --cross --nq 1100 2>&1 | grep attn_train
