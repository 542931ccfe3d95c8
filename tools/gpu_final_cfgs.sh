#!/bin/bash
# round-3 final: other workloads, config-5 rank shape, 1-rank sharded bench, 8-rank simulations
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=$1; O=gpurun_out/$T; mkdir -p $O
for c in ecoli1m yeast5m ecoli10m_err genome200m_k51_r8; do
  s=10; [ $c = genome200m_k51_r8 ] && s=3
  timeout -k 10 400 python bench.py --config $c --steps $s --warmup 2 --no-cpu-baseline --no-host-input > $O/$c.json 2> $O/$c.err || { echo $c FAILED; tail -20 $O/$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$c.json'));print('$c', d['ms_per_step'], d['stage_ms'])"
done
timeout -k 10 300 python bench.py --sharded --steps 10 --warmup 3 --no-cpu-baseline --no-host-input > $O/sharded1.json 2> $O/sharded1.err || { echo SHARDED FAILED; tail -20 $O/sharded1.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/sharded1.json'));print('sharded1', d['ms_per_step'], d['sharded_phase_ms'])"
timeout -k 10 400 python -u tools/sim_sharded.py --ranks 8 --weak > $O/sim8_weak.log 2>&1 || { echo SIMW FAILED; tail -20 $O/sim8_weak.log; exit 1; }
tail -12 $O/sim8_weak.log
timeout -k 10 300 python -u tools/sim_sharded.py --ranks 8 > $O/sim8_strong.log 2>&1 || { echo SIMS FAILED; tail -20 $O/sim8_strong.log; exit 1; }
tail -12 $O/sim8_strong.log
