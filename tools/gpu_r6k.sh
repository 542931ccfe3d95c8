#!/bin/bash
# round 6: join_local.h with spread append counters, junction buckets by radix sort, two copy
# streams for host input: tests, kernel traces (headline, config 5's shape), pipelined loop with
# one / two copy streams, config 5's per-rank step, the bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6k}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_assemble_gpu.py tests/test_distributed_gpu.py tests/test_host_input_gpu.py tests/test_host_api_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "join or golden or sk2 or wide or junction or staged or host or pipe or stream" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
NOPMC=1 bash tools/gpu_prof.sh ${T}_prof ecoli10m > $O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof.log; exit 1; }
python3 tools/rocpd_stats.py $O/../${T}_prof/kt/run_results.db $O/headline_kernel_stats.csv && head -16 $O/headline_kernel_stats.csv | cut -c1-60
NOPMC=1 bash tools/gpu_prof.sh ${T}_c5 genome200m_k51_r8 > $O/prof_c5.log 2>&1 || { echo PROF C5 FAILED; tail -20 $O/prof_c5.log; exit 1; }
python3 tools/rocpd_stats.py $O/../${T}_c5/kt/run_results.db $O/c5_kernel_stats.csv && head -16 $O/c5_kernel_stats.csv | cut -c1-60
grep -h '"stage_ms"' $O/../${T}_prof/bench_kt.json $O/../${T}_c5/bench_kt.json | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['stage_ms']) for l in sys.stdin]"
timeout -k 10 300 python3 tools/pipe_trace.py 10 > $O/pipe2.log 2>&1 || { echo PIPE FAILED; tail -20 $O/pipe2.log; exit 1; }
grep pipelined $O/pipe2.log
EULERHIP_COPY_STREAMS=1 timeout -k 10 300 python3 tools/pipe_trace.py 10 > $O/pipe1.log 2>&1 || { echo PIPE1 FAILED; tail -20 $O/pipe1.log; exit 1; }
grep pipelined $O/pipe1.log
timeout -k 10 600 python -u tools/sim_sharded.py --ranks 1 --reads 12500000 --genome 200000000 --len 150 --k 51 --reps 3 --read-base 37500000 --seed 20261020 > $O/c5_rank_sharded.log 2>&1 || { echo C5 SHARDED FAILED; tail -30 $O/c5_rank_sharded.log; exit 1; }
grep "rep .*max\|HBM" $O/c5_rank_sharded.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_full.json 2> $O/bench_full.err || { echo BENCH FAILED; tail -20 $O/bench_full.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('headline', d['ms_per_step'], d['roofline']['frac'], d['host_input']['ms_per_step'], d['host_input']['pipelined'], d['host_input']['h2d_ms'])" $O/bench_full.json
