#!/bin/bash
# A/B of debug knobs on a bench config (CFG, default the headline): gpu_ab.sh TAG "name:ENV=v ENV2=v" ...
# (2 reps each, interleaved); prints ms/step and the stages per variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=$1; shift
B="bench.py --config ${CFG:-ecoli10m} --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-host-input"
for rep in 1 2; do
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    env EULERHIP_DEBUG=1 $envs timeout -k 10 200 python $B > gpurun_out/${T}_${name}_$rep.json 2> gpurun_out/${T}_${name}_$rep.err || { echo BENCH FAILED $name; tail -20 gpurun_out/${T}_${name}_$rep.err; exit 1; }
  done
done
T=$T python3 - <<'PY'
import json,glob,os
for f in sorted(glob.glob('gpurun_out/'+os.environ['T']+'_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d['ms_per_step'], {k: v for k, v in d['stage_ms'].items() if v > 0.05})
PY
