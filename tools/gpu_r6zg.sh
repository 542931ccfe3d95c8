#!/bin/bash
# round 6: starts filter with its loads issued together -- one-GPU assembly tests, headline kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6zg}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_assemble_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
NOPMC=1 bash tools/gpu_prof.sh ${T}_prof ecoli10m > $O/prof.log 2>&1 || { echo PROF FAILED; tail -20 $O/prof.log; exit 1; }
grep -h '"stage_ms"' gpurun_out/${T}_prof/bench_kt.json | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['stage_ms']) for l in sys.stdin]"
grep "k_starts_count\|k_starts_write" gpurun_out/${T}_prof/kernel_stats.csv | cut -d, -f1,3-5 | cut -c1-60,200-
