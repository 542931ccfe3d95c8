#!/bin/bash
# rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes of the headline bench (gpurun_out/TAG_*)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-prof}; CFG=${2:-ecoli10m}
O=gpurun_out/$TAG; mkdir -p $O
B="bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-host-input"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 $B > $O/bench_kt.json 2> $O/kt.err || { echo KT FAILED; tail -20 $O/kt.err; exit 1; }
cat $O/bench_kt.json
if [ -z "$NOPMC" ]; then
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run -- python3 $B > /dev/null 2> $O/fetch.err || { echo FETCH FAILED; tail -5 $O/fetch.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run -- python3 $B > /dev/null 2> $O/write.err || { echo WRITE FAILED; tail -5 $O/write.err; exit 1; }
echo PMC done
WL=$(python3 -c "import sys; sys.path.insert(0, '.'); import bench; print(bench.CONFIGS['$CFG']['name'])")
python3 profiles/collect_traffic.py $O/fetch $O/write "$WL" ${TAG} > $O/traffic.json 2> $O/traffic.err || true
fi
python3 tools/rocpd_stats.py $O/kt/run_results.db $O/kernel_stats.csv || true
# (the databases stay on the box: a call's gpurun_out is merged back only below 64 MiB)
[ -n "$KEEPDB" ] || rm -rf $O/kt $O/fetch $O/write
