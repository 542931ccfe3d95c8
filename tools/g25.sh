set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g25; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py tests/test_assemble_gpu.py tests/test_host_api_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && python -c "import json;d=json.load(open('$O/bench.json'));print(d['ms_per_step'], d['stage_ms'])"

