set -uo pipefail
OUT=gpurun_out/r6g; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for g in 0 1 0 1; do
CMT_TRAIN_GRAPH=$g timeout -k 10 300 python3 -u bench.py --train --workload coop --steps 30 --warmup 5 > $OUT/train_g$g.json 2> $OUT/train_g$g.log || { echo "train failed"; tail $OUT/train_g$g.log; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/train_g$g.json')); print('graph', $g, d['value'], d['ms_per_step'])"
done
