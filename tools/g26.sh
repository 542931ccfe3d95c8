set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g26; mkdir -p $O
timeout -k 10 400 python bench.py --config genome20m_k51 --no-cpu-baseline --steps 3 > $O/bench51.json 2> $O/bench51.err && python -c "import json;d=json.load(open('$O/bench51.json'));print(d['ms_per_step'], d['value'], d['stage_ms'], d['roofline']['kernels_ms'], d['config'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python3 bench.py --config genome20m_k51 --no-cpu-baseline --steps 2 --warmup 1 > $O/ks.log 2>&1
