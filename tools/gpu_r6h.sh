#!/bin/bash
# round 6: exact-size partitioned outputs + free-memory-aware trims (GPU tests of the sharded /
# partitioned / host-input paths, config 5's per-rank step three times with the allocation log),
# the bench line (host input collapsed when the staged copy is complete), then the r6g profiles
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6h}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sharded or partition or place or staged or host or junction or distributed or stream" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
EULERHIP_MEMLOG=1 timeout -k 10 600 python -u tools/sim_sharded.py --ranks 1 --reads 12500000 --genome 200000000 --len 150 --k 51 --reps 3 --read-base 37500000 --seed 20261020 > $O/c5_rank_sharded.log 2>&1 || { echo C5 SHARDED FAILED; grep -v "eulerhip mem" $O/c5_rank_sharded.log | tail -30; exit 1; }
grep "rep \|count per" $O/c5_rank_sharded.log | grep -v median
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_full.json 2> $O/bench_full.err || { echo BENCH FAILED; tail -20 $O/bench_full.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('headline', d['ms_per_step'], d['host_input']['ms_per_step'], d['host_input']['pipelined'], d['host_input']['h2d_ms'])" $O/bench_full.json
bash tools/gpu_r6g.sh ${T}g
