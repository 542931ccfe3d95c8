#!/bin/bash
# round 6 profiles: kernel stats + FETCH / WRITE passes of the headline and of config 5's rank
# shape, SQ counters of the headline (three passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6g}
bash tools/gpu_prof.sh ${T}_prof ecoli10m || exit 1
bash tools/gpu_prof.sh ${T}_c5 genome200m_k51_r8 || exit 1
bash profiles/pmc_default.sh gpurun_out/${T}_sq || { echo SQ FAILED; exit 1; }
head -60 gpurun_out/${T}_sq/summary.txt
