#!/bin/bash
# round 6: the 4-wave k_skpart_w (tests + headline bench), then config 5's per-rank sharded step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6b}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_assemble_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_assemble.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests_assemble.log; exit 1; }
tail -2 $O/tests_assemble.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-input > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail -20 $O/bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('headline', d['ms_per_step'], d['stage_ms'], d['roofline']['kernels_ms'])" $O/bench.json
EULERHIP_MEMLOG=1 timeout -k 10 400 python -u tools/sim_sharded.py --ranks 1 --reads 12500000 --genome 200000000 --len 150 --k 51 --reps 2 --read-base 37500000 --seed 20261020 > $O/c5_rank_sharded.log 2>&1 || { echo C5 SHARDED FAILED; grep -v "eulerhip mem" $O/c5_rank_sharded.log | tail -30; exit 1; }
grep -v "eulerhip mem" $O/c5_rank_sharded.log | tail -8
timeout -k 10 500 python -u -m pytest tests/test_configs_gpu.py -x -q -s --timeout 450 --timeout-method thread -k "config5_rank_sharded" > $O/tests_c5.log 2>&1 || { echo C5 TEST FAILED; tail -30 $O/tests_c5.log; exit 1; }
grep -E "config-5|passed|failed" $O/tests_c5.log | tail -3
