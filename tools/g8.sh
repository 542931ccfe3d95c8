set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g8; mkdir -p $O
EULERHIP_BUCKET12=2 timeout -k 10 400 python -u -m pytest tests/test_assemble_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && python -c "import json;d=json.load(open('$O/bench.json'));print(d['ms_per_step'], d['roofline']['kernels_ms'])"
EULERHIP_BUCKET12=2 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench12.json 2> $O/bench12.err && python -c "import json;d=json.load(open('$O/bench12.json'));print(d['ms_per_step'], d['roofline']['kernels_ms'])"
