set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g16; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log
bash profiles/profile_round.sh gpurun_out/g16/prof && cat gpurun_out/g16/prof/bench.json
