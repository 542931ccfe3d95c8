#!/bin/bash
# round 6: the full GPU suite and smoke on the current tree, then the multi-GPU sims (runs gather
# as shipped) and config 5's per-rank step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6o}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || { echo SUITE FAILED; tail -40 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --weak --reps 3 > $O/sim8_weak.log 2>&1 || { echo SIM8W FAILED; tail -20 $O/sim8_weak.log; exit 1; }
tail -3 $O/sim8_weak.log | cut -c1-420
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --reps 3 > $O/sim8_strong.log 2>&1 || { echo SIM8S FAILED; tail -20 $O/sim8_strong.log; exit 1; }
tail -3 $O/sim8_strong.log | cut -c1-420
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --reads 10000000 --genome 20000000 --len 150 --k 51 --reps 3 > $O/sim8_k51_genome20m.log 2>&1 || { echo SIM8K51 FAILED; tail -20 $O/sim8_k51_genome20m.log; exit 1; }
tail -3 $O/sim8_k51_genome20m.log | cut -c1-420
timeout -k 10 600 python -u tools/sim_sharded.py --ranks 1 --reads 12500000 --genome 200000000 --len 150 --k 51 --reps 3 --read-base 37500000 --seed 20261020 > $O/c5_rank_sharded.log 2>&1 || { echo C5 SHARDED FAILED; tail -30 $O/c5_rank_sharded.log; exit 1; }
grep "rep .*max\|HBM" $O/c5_rank_sharded.log | cut -c1-420
