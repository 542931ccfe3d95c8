#!/bin/bash
# round 6: multi-GPU sims (weak / strong 8 ranks at the headline, 8 ranks k = 51 on the junction
# flow), config 5's one-rank sharded step twice, 20 M reads of config 5 on one GPU (streaming and
# one-shot), the pipelined host-input loop traced, the full bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6f}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --weak --reps 3 > $O/sim8_weak.log 2>&1 || { echo SIM8W FAILED; tail -20 $O/sim8_weak.log; exit 1; }
tail -3 $O/sim8_weak.log
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --reps 3 > $O/sim8_strong.log 2>&1 || { echo SIM8S FAILED; tail -20 $O/sim8_strong.log; exit 1; }
tail -3 $O/sim8_strong.log
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --reads 10000000 --genome 20000000 --len 150 --k 51 --reps 3 > $O/sim8_k51_genome20m.log 2>&1 || { echo SIM8K51 FAILED; tail -20 $O/sim8_k51_genome20m.log; exit 1; }
tail -3 $O/sim8_k51_genome20m.log
timeout -k 10 600 python -u tools/sim_sharded.py --ranks 1 --reads 12500000 --genome 200000000 --len 150 --k 51 --reps 2 --read-base 37500000 --seed 20261020 > $O/c5_rank_sharded.log 2>&1 || { echo C5 SHARDED FAILED; tail -30 $O/c5_rank_sharded.log; exit 1; }
tail -4 $O/c5_rank_sharded.log
timeout -k 10 600 python -u tools/stream_rank.py --reads 20000000 --chunk 5000000 --fold 2 --oneshot > $O/stream_20m.log 2>&1 || { echo STREAM20 FAILED; tail -20 $O/stream_20m.log; exit 1; }
tail -3 $O/stream_20m.log
mkdir -p $O/pipe
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/pipe -o run -- python3 tools/pipe_trace.py 10 > $O/pipe_trace.log 2>&1 || { echo PIPE TRACE FAILED; tail -20 $O/pipe_trace.log; exit 1; }
grep pipelined $O/pipe_trace.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_full.json 2> $O/bench_full.err || { echo BENCH FAILED; tail -20 $O/bench_full.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('headline', d['ms_per_step'], d['host_input']['ms_per_step'], d['host_input']['pipelined'], d['host_input']['h2d_ms'])" $O/bench_full.json
