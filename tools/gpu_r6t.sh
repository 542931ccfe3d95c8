#!/bin/bash
# round 6: k_skbucket3 record table 1664 vs 1280 entries (EULERHIP_SK2_B3_RS, four workgroups a
# CU): distinct-record statistics, parity of the super-k-mer tests with 1280, step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6t}
O=gpurun_out/$T; mkdir -p $O
for cfg in ecoli10m; do
EULERHIP_DEBUG=1 EULERHIP_SK2_STATS=1 timeout -k 10 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-host-input > /dev/null 2> $O/stats_$cfg.err || { echo STATS FAILED; tail -20 $O/stats_$cfg.err; exit 1; }
grep "k_skbucket3:\|count_sk2" $O/stats_$cfg.err | sort | uniq -c | head -5
done
EULERHIP_SK2_B3_RS=1280 timeout -k 10 900 python -u -m pytest tests/test_assemble_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sk2 or golden or ecoli10m or rank_sizes or starts_small" > $O/tests1280.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests1280.log; exit 1; }
tail -2 $O/tests1280.log
for rs in 1664 1280 1664 1280; do
EULERHIP_DEBUG=1 EULERHIP_SK2_B3_RS=$rs timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-input > $O/b_$rs.json 2> $O/b_$rs.err || { echo BENCH FAILED; tail -20 $O/b_$rs.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rs', sys.argv[2], d['ms_per_step'], 'compact', d['stage_ms']['compact'], d['roofline']['kernels_ms'])" $O/b_$rs.json $rs
done
