#!/bin/bash
# round 6: same-box A/B of the headline bench, the r06_y tree (_ab_old, built in a temporary
# worktree) against this tree, alternated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r6zi}
O=$PWD/gpurun_out/$T; mkdir -p $O
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-input"
for i in 1 2; do
  (cd _ab_old && timeout -k 10 300 python $B > $O/old_$i.json 2> $O/old_$i.err) || { echo OLD FAILED; tail -20 $O/old_$i.err; exit 1; }
  timeout -k 10 300 python $B > $O/new_$i.json 2> $O/new_$i.err || { echo NEW FAILED; tail -20 $O/new_$i.err; exit 1; }
done
for f in old_1 new_1 old_2 new_2; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['ms_per_step'], r['kernels_ms'])" $O/$f.json $f; done
