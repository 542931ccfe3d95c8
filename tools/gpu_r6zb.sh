#!/bin/bash
# round 6: ruler-state spare on first allocation -- partitioned tests, the weak / strong 8-rank sims
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6zb}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "partition or sharded" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --weak --reps 4 > $O/sim8_weak.log 2>&1 || { echo SIM8W FAILED; tail -20 $O/sim8_weak.log; exit 1; }
grep "rep .*max\|HBM" $O/sim8_weak.log | cut -c1-330
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --reps 4 > $O/sim8_strong.log 2>&1 || { echo SIM8S FAILED; tail -20 $O/sim8_strong.log; exit 1; }
grep "rep .*max\|HBM" $O/sim8_strong.log | cut -c1-330
