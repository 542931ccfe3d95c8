#!/bin/bash
# round 6: kernel stats + FETCH / WRITE traffic of the current build (headline, config 5's shape;
# summarised on the box), then the bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6n}
O=gpurun_out/$T; mkdir -p $O
bash tools/gpu_prof.sh ${T}_prof ecoli10m > $O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof.log; exit 1; }
bash tools/gpu_prof.sh ${T}_c5 genome200m_k51_r8 > $O/prof_c5.log 2>&1 || { echo PROF C5 FAILED; tail -20 $O/prof_c5.log; exit 1; }
grep -h '"stage_ms"' $O/../${T}_prof/bench_kt.json $O/../${T}_c5/bench_kt.json | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['stage_ms']) for l in sys.stdin]"
head -5 $O/../${T}_prof/kernel_stats.csv | cut -c1-80
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_full.json 2> $O/bench_full.err || { echo BENCH FAILED; tail -20 $O/bench_full.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('headline', d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic_source'], d['host_input']['ms_per_step'], d['host_input']['pipelined'], d['host_input']['h2d_ms'])" $O/bench_full.json
