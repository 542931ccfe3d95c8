set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g31; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_assemble_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "synthetic or golden" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in ecoli10m ecoli10m_err; do timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 1; python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', d['ms_per_step'], d['stage_ms'])"; done
