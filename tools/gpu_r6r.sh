#!/bin/bash
# round 6: the local join's gate fallbacks, then the join / golden / wide tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6r}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_assemble_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "join or golden or wide or rank" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
grep -c "gate_falls_back" $O/tests.log || true
