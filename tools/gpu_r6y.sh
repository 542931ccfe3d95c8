#!/bin/bash
# round 6 final tree (A): the full GPU suite, smoke, the bench line, error-rich and config-5 shape
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6y}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || { echo SUITE FAILED; tail -40 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH FAILED; tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('headline', d['ms_per_step'], d['stage_ms'], d['roofline']['frac'], d['host_input']['ms_per_step'], d['host_input']['pipelined']['ms_per_step'])" $O/bench_default.json
timeout -k 10 300 python bench.py --config ecoli10m_err --steps 10 --warmup 3 --no-cpu-baseline --no-host-input > $O/ecoli10m_err.json 2> $O/ecoli10m_err.err || { echo ERR BENCH FAILED; tail -20 $O/ecoli10m_err.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('error-rich', d['ms_per_step'])" $O/ecoli10m_err.json
timeout -k 10 300 python bench.py --config genome200m_k51_r8 --steps 5 --warmup 2 --no-cpu-baseline --no-host-input > $O/config5_shape.json 2> $O/config5_shape.err || { echo C5 BENCH FAILED; tail -20 $O/config5_shape.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('config5 shape', d['ms_per_step'], d['stage_ms'])" $O/config5_shape.json
