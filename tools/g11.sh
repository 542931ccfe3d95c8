set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g11; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench0.json 2> $O/bench0.err && python -c "import json;d=json.load(open('$O/bench0.json'));print(0, d['ms_per_step'], d['roofline']['kernels_ms'])" || exit 1
EULERHIP_X16=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench1.json 2> $O/bench1.err && python -c "import json;d=json.load(open('$O/bench1.json'));print(1, d['ms_per_step'], d['roofline']['kernels_ms'], d['config']['contigs'])" || exit 1
