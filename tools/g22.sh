set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g22; mkdir -p $O
for n in 2 4 8; do timeout -k 10 200 python tools/sim_sharded.py --ranks $n > $O/sim$n.log 2>&1 || exit 1; tail -3 $O/sim$n.log; done
