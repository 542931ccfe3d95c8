#!/bin/bash
# round 6: full GPU suite on the 4-wave partition, the 8-rank k = 51 sim on the junction flow
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6c}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 450 --timeout-method thread > $O/gpu_suite.log 2>&1 || { echo SUITE FAILED; tail -30 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --reads 10000000 --genome 20000000 --len 150 --k 51 --reps 3 > $O/sim8_k51_genome20m.log 2>&1 || { echo SIM8 FAILED; tail -30 $O/sim8_k51_genome20m.log; exit 1; }
tail -5 $O/sim8_k51_genome20m.log
