#!/bin/bash
# round 6: tests touched by PathOf / k_bucket_wr / the wide merge sizing; config-5 shape A/B
# (two k_bucket_wr workgroups a CU vs one), streaming and one-rank sharded config 5 with HBM peaks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6e}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_assemble_gpu.py tests/test_distributed_gpu.py tests/test_configs_gpu.py -x -q --timeout 450 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "^E |FAILED" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-input > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail -20 $O/bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('headline', d['ms_per_step'], d['stage_ms'], d['roofline']['kernels_ms'])" $O/bench.json
for v in 0 1; do
EULERHIP_DEBUG=1 EULERHIP_WR_ONE=$v timeout -k 10 300 python bench.py --config genome200m_k51_r8 --steps 5 --warmup 2 --no-cpu-baseline --no-host-input > $O/c5_wrone$v.json 2> $O/c5_wrone$v.err || { echo C5 FAILED; tail -20 $O/c5_wrone$v.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5 wr_one=$v', d['ms_per_step'], d['stage_ms'], d['config']['hbm_used_gb'])" $O/c5_wrone$v.json
done
timeout -k 10 600 python -u tools/stream_rank.py --chunk 4000000 --fold 2 > $O/stream_rank.log 2>&1 || { echo STREAM FAILED; tail -20 $O/stream_rank.log; exit 1; }
tail -2 $O/stream_rank.log
timeout -k 10 600 python -u tools/sim_sharded.py --ranks 1 --reads 12500000 --genome 200000000 --len 150 --k 51 --reps 2 --read-base 37500000 --seed 20261020 > $O/c5_rank_sharded.log 2>&1 || { echo C5 SHARDED FAILED; tail -30 $O/c5_rank_sharded.log; exit 1; }
tail -4 $O/c5_rank_sharded.log
