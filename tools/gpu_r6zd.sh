#!/bin/bash
# round 6: the partitioned finish's chain records in the placed segment's junction-slot buffer --
# sharded / partitioned GPU tests, config 5's per-rank step with the allocation log, the 20 M-read
# streaming run, the weak 8-rank sim
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6zd}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sharded or partition or place or junction or distributed or stream or rank" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
EULERHIP_MEMLOG=1 timeout -k 10 600 python -u tools/sim_sharded.py --ranks 1 --reads 12500000 --genome 200000000 --len 150 --k 51 --reps 2 --read-base 37500000 --seed 20261020 > $O/c5_rank_sharded.log 2>&1 || { echo C5 SHARDED FAILED; grep -v "eulerhip mem" $O/c5_rank_sharded.log | tail -30; exit 1; }
grep "rep .*max\|HBM" $O/c5_rank_sharded.log | cut -c1-420
timeout -k 10 600 python -u tools/stream_rank.py --reads 20000000 --chunk 5000000 --fold 2 --oneshot > $O/stream_20m.log 2>&1 || { echo STREAM20 FAILED; tail -20 $O/stream_20m.log; exit 1; }
tail -3 $O/stream_20m.log
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --weak --reps 3 > $O/sim8_weak.log 2>&1 || { echo SIM8W FAILED; tail -20 $O/sim8_weak.log; exit 1; }
grep "rep .*max\|HBM" $O/sim8_weak.log | cut -c1-330
