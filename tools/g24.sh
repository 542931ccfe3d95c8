set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g24; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py tests/test_assemble_gpu.py tests/test_cli_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/sim_sharded.py --ranks 8 > $O/sim8.log 2>&1 && tail -3 $O/sim8.log
