#!/bin/bash
# round 6: k_tile_chains at 40 KB (four workgroups a CU) -- ranking / golden / sharded / config
# tests, kernel traces of the headline and config 5's shape, the bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6s}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_assemble_gpu.py tests/test_distributed_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rank or golden or partition or sharded or starts or err or genome20m or config5 or wide" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
NOPMC=1 bash tools/gpu_prof.sh ${T}_prof ecoli10m > $O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof.log; exit 1; }
NOPMC=1 bash tools/gpu_prof.sh ${T}_c5 genome200m_k51_r8 > $O/prof_c5.log 2>&1 || { echo PROF C5 FAILED; tail -20 $O/prof_c5.log; exit 1; }
grep -h '"stage_ms"' $O/../${T}_prof/bench_kt.json $O/../${T}_c5/bench_kt.json | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['stage_ms']) for l in sys.stdin]"
grep -h "tile_chains" $O/../${T}_prof/kernel_stats.csv $O/../${T}_c5/kernel_stats.csv | cut -d, -f2- | cut -c1-200 | awk -F, '{print $(NF-5), $(NF-3)}'
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_full.json 2> $O/bench_full.err || { echo BENCH FAILED; tail -20 $O/bench_full.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('headline', d['ms_per_step'], d['stage_ms']['rank'], d['roofline']['frac'], d['host_input']['ms_per_step'], d['host_input']['pipelined']['ms_per_step'])" $O/bench_full.json
