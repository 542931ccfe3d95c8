#!/bin/bash
# round 6: local-join setup in one launch -- join tests, the bench line, kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6v}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_assemble_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "join or golden or ecoli10m or genome20m or sk2" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_full.json 2> $O/bench_full.err || { echo BENCH FAILED; tail -20 $O/bench_full.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('headline', d['ms_per_step'], d['stage_ms'], d['roofline']['frac'], d['host_input']['ms_per_step'], d['host_input']['pipelined']['ms_per_step'])" $O/bench_full.json
timeout -k 10 300 python bench.py --config ecoli10m_err --steps 10 --warmup 3 --no-cpu-baseline --no-host-input > $O/ecoli10m_err.json 2> $O/ecoli10m_err.err || { echo ERR BENCH FAILED; tail -20 $O/ecoli10m_err.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('error-rich', d['ms_per_step'], d['stage_ms'])" $O/ecoli10m_err.json
