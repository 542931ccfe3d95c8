set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g10; mkdir -p $O
for v in 1024 2048 4096 8192; do EULERHIP_MAX_GROUPS=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench$v.json 2> $O/bench$v.err && python -c "import json;d=json.load(open('$O/bench$v.json'));print($v, d['ms_per_step'], d['roofline']['kernels_ms'], d['stage_ms'])" || exit 1; done
