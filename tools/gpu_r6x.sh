#!/bin/bash
# round 6: run codes from k_wbv's 2-bit reads, the run upsweep with eight loads in flight --
# 128-bit tests, config 5's shape traced, packed / ASCII A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6x}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_assemble_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "wide or genome20m or config5 or 51 or 45 or golden or stream" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
NOPMC=1 bash tools/gpu_prof.sh ${T}_c5 genome200m_k51_r8 > $O/prof_c5.log 2>&1 || { echo PROF C5 FAILED; tail -20 $O/prof_c5.log; exit 1; }
grep -h '"stage_ms"' $O/../${T}_c5/bench_kt.json | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['stage_ms']) for l in sys.stdin]"
grep -h "upsweep\|k_wbv\|run_codes" $O/../${T}_c5/kernel_stats.csv | python3 -c "import sys,csv; [print(r[0].split('(')[0], round(float(r[3])/1e3,1)) for r in csv.reader(sys.stdin)]"
for pk in 0 1 0 1; do
EULERHIP_DEBUG=1 EULERHIP_RUN_PACKED=$pk timeout -k 10 300 python bench.py --config genome200m_k51_r8 --steps 3 --warmup 1 --no-cpu-baseline --no-host-input > $O/c5_$pk.json 2> $O/c5_$pk.err || { echo C5 BENCH FAILED; tail -20 $O/c5_$pk.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('packed', sys.argv[2], d['ms_per_step'], d['stage_ms']['prescan'], d['stage_ms']['compact'])" $O/c5_$pk.json $pk
done
