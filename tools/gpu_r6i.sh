#!/bin/bash
# round 6: the local junction join (join_local.h) against the oracle, then measured (headline
# and config 5's shape, kernel trace), config 5's per-rank step three times, the pipelined
# host-input loop traced
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6i}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_assemble_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "join or golden or sk2 or wide" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
NOPMC=1 bash tools/gpu_prof.sh ${T}_prof ecoli10m > $O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof.log; exit 1; }
python3 tools/rocpd_stats.py $O/../${T}_prof/kt/run_results.db $O/headline_kernel_stats.csv && head -14 $O/headline_kernel_stats.csv | cut -c1-60
NOPMC=1 bash tools/gpu_prof.sh ${T}_c5 genome200m_k51_r8 > $O/prof_c5.log 2>&1 || { echo PROF C5 FAILED; tail -20 $O/prof_c5.log; exit 1; }
python3 tools/rocpd_stats.py $O/../${T}_c5/kt/run_results.db $O/c5_kernel_stats.csv && head -20 $O/c5_kernel_stats.csv | cut -c1-60
grep -h '"stage_ms"' $O/../${T}_prof/bench_kt.json $O/../${T}_c5/bench_kt.json | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['stage_ms']) for l in sys.stdin]"
EULERHIP_MEMLOG=1 timeout -k 10 600 python -u tools/sim_sharded.py --ranks 1 --reads 12500000 --genome 200000000 --len 150 --k 51 --reps 3 --read-base 37500000 --seed 20261020 > $O/c5_rank_sharded.log 2>&1 || { echo C5 SHARDED FAILED; grep -v "eulerhip mem" $O/c5_rank_sharded.log | tail -30; exit 1; }
grep "rep .*max\|HBM" $O/c5_rank_sharded.log
mkdir -p $O/pipe
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/pipe -o run -- python3 tools/pipe_trace.py 10 > $O/pipe_trace.log 2>&1 || { echo PIPE TRACE FAILED; tail -20 $O/pipe_trace.log; exit 1; }
grep pipelined $O/pipe_trace.log
