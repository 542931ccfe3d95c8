#!/bin/bash
# round 6: join_local.h without scratch (scan fused with the run bounds) against the oracle and
# timed (headline + config 5's shape); the pipelined host-input loop with SDMA copies and with
# blit-kernel copies (HSA_ENABLE_SDMA=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6j}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_assemble_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "join or golden or sk2 or wide" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
NOPMC=1 bash tools/gpu_prof.sh ${T}_prof ecoli10m > $O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof.log; exit 1; }
python3 tools/rocpd_stats.py $O/../${T}_prof/kt/run_results.db $O/headline_kernel_stats.csv && head -14 $O/headline_kernel_stats.csv | cut -c1-60
NOPMC=1 bash tools/gpu_prof.sh ${T}_c5 genome200m_k51_r8 > $O/prof_c5.log 2>&1 || { echo PROF C5 FAILED; tail -20 $O/prof_c5.log; exit 1; }
python3 tools/rocpd_stats.py $O/../${T}_c5/kt/run_results.db $O/c5_kernel_stats.csv && head -14 $O/c5_kernel_stats.csv | cut -c1-60
grep -h '"stage_ms"' $O/../${T}_prof/bench_kt.json $O/../${T}_c5/bench_kt.json | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['stage_ms']) for l in sys.stdin]"
timeout -k 10 300 python3 tools/pipe_trace.py 10 > $O/pipe_sdma.log 2>&1 || { echo PIPE FAILED; tail -20 $O/pipe_sdma.log; exit 1; }
grep pipelined $O/pipe_sdma.log
HSA_ENABLE_SDMA=0 timeout -k 10 300 python3 tools/pipe_trace.py 10 > $O/pipe_blit.log 2>&1 || { echo PIPE BLIT FAILED; tail -20 $O/pipe_blit.log; exit 1; }
grep pipelined $O/pipe_blit.log
mkdir -p $O/pipe_blit
HSA_ENABLE_SDMA=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/pipe_blit -o run -- python3 tools/pipe_trace.py 10 > $O/pipe_blit_trace.log 2>&1 || { echo PIPE BLIT TRACE FAILED; tail -20 $O/pipe_blit_trace.log; exit 1; }
grep pipelined $O/pipe_blit_trace.log
