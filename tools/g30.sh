set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g30; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_assemble_gpu.py tests/test_host_api_gpu.py tests/test_cli_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python bench.py --config ecoli10m_err --no-cpu-baseline > $O/bench_err.json 2> $O/bench_err.err && python -c "import json;d=json.load(open('$O/bench_err.json'));print(d['ms_per_step'], '%.3g'%d['value'], d['stage_ms'], d['roofline']['kernels_ms'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python3 bench.py --config ecoli10m_err --no-cpu-baseline --steps 2 --warmup 1 > $O/ks.log 2>&1
