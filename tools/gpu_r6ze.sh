#!/bin/bash
# round 6: config 5's per-rank step, three steps with the allocation log (steady-state check)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6ze}
O=gpurun_out/$T; mkdir -p $O
EULERHIP_MEMLOG=1 timeout -k 10 600 python -u tools/sim_sharded.py --ranks 1 --reads 12500000 --genome 200000000 --len 150 --k 51 --reps 3 --read-base 37500000 --seed 20261020 > $O/c5_rank_sharded.log 2>&1 || { echo C5 SHARDED FAILED; grep -v "eulerhip mem" $O/c5_rank_sharded.log | tail -30; exit 1; }
grep "rep .*max\|HBM" $O/c5_rank_sharded.log | cut -c1-300
