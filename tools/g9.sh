set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g9; mkdir -p $O
EULERHIP_BUCKET12=2 timeout -k 10 400 python -u -m pytest tests/test_assemble_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 0 1 2; do EULERHIP_BUCKET12=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench$v.json 2> $O/bench$v.err && python -c "import json;d=json.load(open('$O/bench$v.json'));print($v, d['ms_per_step'], d['roofline']['kernels_ms'])" || exit 1; done
