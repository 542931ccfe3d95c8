#!/bin/bash
# round 6, first GPU pass: junction-join split tests, config-5 per-rank sharded step (world 1)
# with HBM accounting, the 8-rank k = 51 sim on the junction flow, config-5 shape allocations
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6a}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_distributed_gpu.py -x -q --timeout 200 --timeout-method thread -k "junction_join_split or partitioned_finish_equals" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
EULERHIP_MEMLOG=1 timeout -k 10 400 python -u tools/sim_sharded.py --ranks 1 --reads 12500000 --genome 200000000 --len 150 --k 51 --reps 2 --read-base 37500000 --seed 20261020 > $O/c5_rank_sharded.log 2>&1 || { echo C5 SHARDED FAILED; tail -30 $O/c5_rank_sharded.log; exit 1; }
grep -v "eulerhip mem" $O/c5_rank_sharded.log | tail -8
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --reads 10000000 --genome 20000000 --len 150 --k 51 --reps 3 > $O/sim8_k51_genome20m.log 2>&1 || { echo SIM8 FAILED; tail -30 $O/sim8_k51_genome20m.log; exit 1; }
tail -4 $O/sim8_k51_genome20m.log
EULERHIP_MEMLOG=1 timeout -k 10 300 python bench.py --config genome200m_k51_r8 --steps 3 --warmup 1 --no-cpu-baseline --no-host-input > $O/c5_shape.json 2> $O/c5_shape.err || { echo C5 SHAPE FAILED; tail -20 $O/c5_shape.err; exit 1; }
grep -c "eulerhip mem" $O/c5_shape.err
