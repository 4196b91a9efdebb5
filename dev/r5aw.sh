#!/bin/bash
# Round-5 step aw: Python GC during the coop training step (default / frozen after warm-up / off).
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
    for m in default freeze disable; do
        GC_MODE=$m timeout -k 10 300 python -u dev/train_gc_probe.py 2>&1 | grep "^gc" || exit 1
    done
done
