#!/bin/bash
# round-4: selected tests (-k SEL) under an extra env assignment (ENV1, optional), then all GPU tests and the bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=$1; SEL=$2
if [ -n "$SEL" ]; then
env $ENV1 timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$SEL" > gpurun_out/${T}_sel.log 2>&1 || { echo SELECTED FAILED; tail -40 gpurun_out/${T}_sel.log; exit 1; }
tail -2 gpurun_out/${T}_sel.log
fi
[ -n "$NOFULL" ] && exit 0
bash tools/gpu_full.sh $T
