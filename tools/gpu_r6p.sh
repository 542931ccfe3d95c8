#!/bin/bash
# round 6: two-hop Wyllie rounds -- ranking / golden / distributed tests, the bench line, the
# error-rich bench, a kernel trace of the headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6p}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_assemble_gpu.py tests/test_distributed_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rank or golden or partition or sharded or starts or err or genome20m" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
NOPMC=1 bash tools/gpu_prof.sh ${T}_prof ecoli10m > $O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof.log; exit 1; }
grep -h '"stage_ms"' $O/../${T}_prof/bench_kt.json | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['stage_ms']) for l in sys.stdin]"
grep -i "rjump\|walk_s\|tile_chains" $O/../${T}_prof/kernel_stats.csv | cut -d, -f2-4 | head
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_full.json 2> $O/bench_full.err || { echo BENCH FAILED; tail -20 $O/bench_full.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('headline', d['ms_per_step'], d['stage_ms']['rank'], d['roofline']['frac'], d['roofline']['traffic_source'], d['host_input']['ms_per_step'], d['host_input']['pipelined']['ms_per_step'], d['host_input']['h2d_ms'])" $O/bench_full.json
timeout -k 10 300 python bench.py --config ecoli10m_err --steps 10 --warmup 3 --no-cpu-baseline --no-host-input > $O/ecoli10m_err.json 2> $O/ecoli10m_err.err || { echo ERR BENCH FAILED; tail -20 $O/ecoli10m_err.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('error-rich', d['ms_per_step'], d['stage_ms'])" $O/ecoli10m_err.json
