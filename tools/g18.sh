set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g18; mkdir -p $O
EULERHIP_LOAD_MERGE=1 timeout -k 10 200 python tools/sim_sharded.py --ranks 8 > $O/sim8.log 2>&1 && tail -4 $O/sim8.log
