set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g15; mkdir -p $O
for v in 5; do EULERHIP_COARSE_BITS=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench$v.json 2> $O/bench$v.err && python -c "import json;d=json.load(open('$O/bench$v.json'));print($v, d['ms_per_step'], d['roofline']['kernels_ms'])" || exit 1; done
