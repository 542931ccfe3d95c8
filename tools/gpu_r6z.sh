#!/bin/bash
# round 6 final tree (B): FETCH / WRITE traffic and kernel stats of the headline and config 5's
# shape, the 8-rank sims, config 5's per-rank step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6z}
O=gpurun_out/$T; mkdir -p $O
bash tools/gpu_prof.sh ${T}_prof ecoli10m > $O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof.log; exit 1; }
bash tools/gpu_prof.sh ${T}_c5 genome200m_k51_r8 > $O/prof_c5.log 2>&1 || { echo PROF C5 FAILED; tail -20 $O/prof_c5.log; exit 1; }
grep -h '"stage_ms"' $O/../${T}_prof/bench_kt.json $O/../${T}_c5/bench_kt.json | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['stage_ms']) for l in sys.stdin]"
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --weak --reps 3 > $O/sim8_weak.log 2>&1 || { echo SIM8W FAILED; tail -20 $O/sim8_weak.log; exit 1; }
tail -3 $O/sim8_weak.log | cut -c1-420
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --reps 3 > $O/sim8_strong.log 2>&1 || { echo SIM8S FAILED; tail -20 $O/sim8_strong.log; exit 1; }
tail -3 $O/sim8_strong.log | cut -c1-420
timeout -k 10 600 python -u tools/sim_sharded.py --ranks 1 --reads 12500000 --genome 200000000 --len 150 --k 51 --reps 2 --read-base 37500000 --seed 20261020 > $O/c5_rank_sharded.log 2>&1 || { echo C5 SHARDED FAILED; tail -30 $O/c5_rank_sharded.log; exit 1; }
grep "rep .*max\|HBM" $O/c5_rank_sharded.log | cut -c1-420
