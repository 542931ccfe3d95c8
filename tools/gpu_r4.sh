#!/bin/bash
# round-4 check: selected tests (-k EXPR, optional), then all GPU tests and the headline bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=$1; SEL=$2
if [ -n "$SEL" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$SEL" > gpurun_out/${T}_sel.log 2>&1 || { echo SELECTED FAILED; tail -40 gpurun_out/${T}_sel.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/${T}_sel.log | tail -20
fi
[ -n "$NOFULL" ] && exit 0
bash tools/gpu_full.sh $T
