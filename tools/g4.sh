set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g4; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_distributed_gpu.py tests/test_assemble_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && cat $O/bench.json
for m in 15 63; do EULERHIP_RULER_MASK=$m timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_m$m.json 2> $O/bench_m$m.err || exit 1; python -c "import json;d=json.load(open('$O/bench_m$m.json'));print($m, d['ms_per_step'], d['stage_ms'])"; done
timeout -k 10 200 python tools/sim_sharded.py --ranks 8 > $O/sim8.log 2>&1 && tail -2 $O/sim8.log
