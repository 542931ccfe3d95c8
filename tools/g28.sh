set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g28; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_assemble_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "filter or synthetic or golden or gfa or links" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python bench.py --config ecoli10m_err --no-cpu-baseline > $O/bench_err.json 2> $O/bench_err.err && python -c "import json;d=json.load(open('$O/bench_err.json'));print(d['ms_per_step'], '%.3g'%d['value'], d['config'], d['stage_ms'], d['roofline']['kernels_ms'])"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && python -c "import json;d=json.load(open('$O/bench.json'));print(d['ms_per_step'], d['stage_ms'])"
