#!/bin/bash
# round-4 SQ counters of the headline bench (three passes, profiles/pmc_default.sh) + kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r4pmc}
bash profiles/pmc_default.sh gpurun_out/$T || { echo PMC FAILED; tail -20 gpurun_out/$T/*.log; exit 1; }
NOPMC=1 bash tools/gpu_prof.sh ${T}_kt ecoli10m
