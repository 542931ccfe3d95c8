#!/bin/bash
# A/B of knob settings on the default bench: each arm twice, interleaved; prints ms_per_step and stages
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=$1; shift
B="bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-input"
for rep in 1 2; do
  i=0
  for arm in "$@"; do
    i=$((i+1))
    env EULERHIP_DEBUG=1 $arm timeout -k 10 200 python $B > gpurun_out/${T}_a${i}_$rep.json 2> gpurun_out/${T}_a${i}_$rep.err || { echo BENCH FAILED $arm; tail -20 gpurun_out/${T}_a${i}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_a${i}_$rep.json').read().strip().splitlines()[-1]); print('$arm', d['ms_per_step'], {k: v for k, v in d['stage_ms'].items() if v > 0.05})"
  done
done
