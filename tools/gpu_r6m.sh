#!/bin/bash
# round 6 (tests first): PMC traffic of the current build (headline, config 5's shape), multi-GPU sims (weak /
# strong 8 ranks, 8 ranks at k = 51), error-rich bench, streaming vs one-shot 20 M reads,
# pipelined loop with one / two copy streams (debug knob)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6m}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_assemble_gpu.py tests/test_distributed_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "join or golden or wide or junction or sharded or partition or genome20m or config5" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_prof.sh ${T}_prof ecoli10m > $O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof.log; exit 1; }
bash tools/gpu_prof.sh ${T}_c5 genome200m_k51_r8 > $O/prof_c5.log 2>&1 || { echo PROF C5 FAILED; tail -20 $O/prof_c5.log; exit 1; }
grep -h '"stage_ms"' $O/../${T}_prof/bench_kt.json $O/../${T}_c5/bench_kt.json | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['stage_ms']) for l in sys.stdin]"
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --weak --reps 3 > $O/sim8_weak.log 2>&1 || { echo SIM8W FAILED; tail -20 $O/sim8_weak.log; exit 1; }
tail -3 $O/sim8_weak.log | cut -c1-400
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --reps 3 > $O/sim8_strong.log 2>&1 || { echo SIM8S FAILED; tail -20 $O/sim8_strong.log; exit 1; }
tail -3 $O/sim8_strong.log | cut -c1-400
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --reads 10000000 --genome 20000000 --len 150 --k 51 --reps 3 > $O/sim8_k51_genome20m.log 2>&1 || { echo SIM8K51 FAILED; tail -20 $O/sim8_k51_genome20m.log; exit 1; }
tail -3 $O/sim8_k51_genome20m.log | cut -c1-400
timeout -k 10 300 python bench.py --config ecoli10m_err --steps 10 --warmup 3 --no-cpu-baseline --no-host-input > $O/ecoli10m_err.json 2> $O/ecoli10m_err.err || { echo ERR BENCH FAILED; tail -20 $O/ecoli10m_err.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('error-rich', d['ms_per_step'], d['stage_ms'])" $O/ecoli10m_err.json
timeout -k 10 600 python -u tools/stream_rank.py --reads 20000000 --chunk 5000000 --fold 2 --oneshot > $O/stream_20m.log 2>&1 || { echo STREAM20 FAILED; tail -20 $O/stream_20m.log; exit 1; }
tail -3 $O/stream_20m.log
for i in 1 2; do
EULERHIP_DEBUG=1 EULERHIP_COPY_STREAMS=1 timeout -k 10 300 python3 tools/pipe_trace.py 10 2>&1 | grep pipelined | sed 's/^/one stream: /'
EULERHIP_DEBUG=1 EULERHIP_COPY_STREAMS=2 timeout -k 10 300 python3 tools/pipe_trace.py 10 2>&1 | grep pipelined | sed 's/^/two streams: /'
done
