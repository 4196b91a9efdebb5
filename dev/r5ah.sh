#!/bin/bash
# Round-5 step ah: host profile of the coop training step (issue vs drain, cProfile, torch op counts).
set -uo pipefail
TAG=${1:-r5ah}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u dev/train_host_profile.py > "$OUT/host.txt" 2> "$OUT/host.log" || { tail "$OUT/host.log"; exit 1; }
grep "issue" "$OUT/host.txt"
