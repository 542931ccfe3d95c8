#!/bin/bash
# round 6: the wide upsweep's HyperLogLog sampled by minimizer -- 128-bit tests, config 5's shape
# traced
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6u}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_assemble_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "wide or genome20m or config5 or 51 or golden or stream" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
NOPMC=1 bash tools/gpu_prof.sh ${T}_c5 genome200m_k51_r8 > $O/prof_c5.log 2>&1 || { echo PROF C5 FAILED; tail -20 $O/prof_c5.log; exit 1; }
grep -h '"stage_ms"' $O/../${T}_c5/bench_kt.json | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['stage_ms']) for l in sys.stdin]"
head -8 $O/../${T}_c5/kernel_stats.csv | cut -c1-70
