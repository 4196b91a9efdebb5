#!/bin/bash
# Full GPU suite + smoke (what the driver runs at round end), logs under gpurun_out/<tag>/.
set -uo pipefail
TAG=${1:-r4s}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > "$OUT/suite.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/suite.log" | tail -3
grep -E "^FAILED|^ERROR" "$OUT/suite.log" | head -20
[[ $rc -eq 0 || $rc -eq 1 ]] || { echo "suite rc=$rc"; tail -20 "$OUT/suite.log"; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -3 "$OUT/smoke.log"
exit $rc
