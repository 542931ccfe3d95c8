set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/g1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g1/pytest.log 2>&1 || { tail -30 gpurun_out/g1/pytest.log; exit 1; }
tail -3 gpurun_out/g1/pytest.log
timeout -k 10 300 python bench.py > gpurun_out/g1/bench.json 2> gpurun_out/g1/bench.err && cat gpurun_out/g1/bench.json
timeout -k 10 300 python bench.py --sharded --no-cpu-baseline > gpurun_out/g1/bench_sh.json 2> gpurun_out/g1/bench_sh.err && cat gpurun_out/g1/bench_sh.json
