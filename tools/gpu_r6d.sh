#!/bin/bash
# round 6: full GPU suite, headline + error-rich benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6d}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 450 --timeout-method thread > $O/gpu_suite.log 2>&1 || { echo SUITE FAILED; grep -E "^E |FAILED|config-5" $O/gpu_suite.log | head -20; tail -5 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-input > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail -20 $O/bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('headline', d['ms_per_step'], d['stage_ms'], d['roofline']['kernels_ms'])" $O/bench.json
timeout -k 10 300 python bench.py --config ecoli10m_err --steps 10 --warmup 3 --no-cpu-baseline --no-host-input > $O/err.json 2> $O/err.err || { echo ERR BENCH FAILED; tail -20 $O/err.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('err', d['ms_per_step'], d['stage_ms'])" $O/err.json
timeout -k 10 600 python -u tools/stream_rank.py --chunk 4000000 --fold 2 --oneshot > $O/stream_rank.log 2>&1 || { echo STREAM FAILED; tail -20 $O/stream_rank.log; exit 1; }
tail -3 $O/stream_rank.log
