#!/bin/bash
# round 6: chain-minimum flag for the starts -- the full GPU suite, smoke, the bench lines
# (gpu_r6y.sh), then the headline's kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r6zf}
bash tools/gpu_r6y.sh $T || exit 1
NOPMC=1 bash tools/gpu_prof.sh ${T}_prof ecoli10m > gpurun_out/$T/prof.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/$T/prof.log; exit 1; }
grep -h '"stage_ms"' gpurun_out/${T}_prof/bench_kt.json | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['stage_ms']) for l in sys.stdin]"
