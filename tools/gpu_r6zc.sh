#!/bin/bash
# round 6: kernel stats of the weak 8-rank sim (which kernels the sharded phases spend on)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6zc}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 -u tools/sim_sharded.py --ranks 8 --weak --reps 3 > $O/sim8_weak.log 2> $O/kt.err || { echo KT FAILED; tail -20 $O/kt.err; exit 1; }
grep "rep .*max" $O/sim8_weak.log | cut -c1-330
python3 tools/rocpd_stats.py $O/kt/run_results.db $O/kernel_stats.csv || true
rm -rf $O/kt
