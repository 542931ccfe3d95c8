set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g23; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --sharded --no-cpu-baseline > $O/bench_sh.json 2> $O/bench_sh.err && python -c "import json;d=json.load(open('$O/bench_sh.json'));print(d['ms_per_step'], d['sharded_phase_ms'])"
timeout -k 10 200 python tools/sim_sharded.py --ranks 8 > $O/sim8.log 2>&1 && tail -3 $O/sim8.log
