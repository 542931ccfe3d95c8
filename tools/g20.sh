set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g20; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench0.json 2> $O/bench0.err && python -c "import json;d=json.load(open('$O/bench0.json'));print('base', d['ms_per_step'], d['roofline']['kernels_ms'])"
EULERHIP_LIB=$GRAFT_REPO_ROOT/pycuda-euler_amd/csrc/build_exp/libeulerhip_exp.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > $O/bench1.json 2> $O/bench1.err; python -c "import json;d=json.load(open('$O/bench1.json'));print('noatomic', d['ms_per_step'], d['roofline']['kernels_ms'])"; tail -3 $O/bench1.err
