#!/bin/bash
# round 6: super-list ruler density A/B (EULERHIP_SRULER_MASK, debug knob) on the headline and
# the error-rich set: step and rank stage
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6q}
O=gpurun_out/$T; mkdir -p $O
for cfg in ecoli10m ecoli10m_err; do
for m in 15 7 3 31 15 7; do
EULERHIP_DEBUG=1 EULERHIP_SRULER_MASK=$m timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-host-input > $O/b_${cfg}_$m.json 2> $O/b_${cfg}_$m.err || { echo BENCH FAILED $cfg $m; tail -20 $O/b_${cfg}_$m.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'mask', sys.argv[3], d['ms_per_step'], 'rank', d['stage_ms']['rank'])" $O/b_${cfg}_$m.json $cfg $m
done
done
