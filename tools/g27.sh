set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g27; mkdir -p $O
for c in ecoli1m yeast5m ecoli10m_err; do timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 1; python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', d['ms_per_step'], '%.3g'%d['value'], d['config']['solid_kmers'], d['config']['buckets'], d['stage_ms'], d['roofline']['kernels_ms'])"; done
