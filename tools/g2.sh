set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g2; mkdir -p $O
timeout -k 10 300 python bench.py --superkmer --no-cpu-baseline > $O/bench_sk.json 2> $O/bench_sk.err && cat $O/bench_sk.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python3 bench.py --superkmer --no-cpu-baseline > $O/ks.log 2>&1
find $O/ks -name '*kernel_stats.csv' | head -1 | xargs cat | cut -c1-200
