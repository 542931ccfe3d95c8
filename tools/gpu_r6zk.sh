#!/bin/bash
# round 6, last tree: the full GPU suite and smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6zk}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || { echo SUITE FAILED; tail -40 $O/gpu_suite.log; exit 1; }
tail -1 $O/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH FAILED; tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('headline', d['ms_per_step'], d['roofline']['frac'], d['host_input']['pipelined']['ms_per_step'])" $O/bench_default.json
