#!/bin/bash
# A/B of knob settings on the error-rich bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=$1; shift
B="bench.py --config ecoli10m_err --steps 10 --warmup 3 --no-cpu-baseline --no-host-input"
i=0
for arm in "$@"; do
  i=$((i+1))
  env EULERHIP_DEBUG=1 $arm timeout -k 10 200 python $B > gpurun_out/${T}_a$i.json 2> gpurun_out/${T}_a$i.err || { echo BENCH FAILED $arm; tail -20 gpurun_out/${T}_a$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_a$i.json').read().strip().splitlines()[-1]); print('$arm', d['ms_per_step'], {k: v for k, v in d['stage_ms'].items() if v > 0.05})"
done
