#!/bin/bash
# A/B PMC passes of the super-k-mer bucket kernel: records merged first (EULERHIP_SK2_DEDUPE=1) or not.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/dd}
mkdir -p $O
for v in 0 1; do
  export EULERHIP_SK2_DEDUPE=$v
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR --output-format csv -d $O/a_$v -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/a_$v.log 2>&1
  timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/b_$v -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/b_$v.log 2>&1
  timeout -k 10 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --output-format csv -d $O/c_$v -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/c_$v.log 2>&1
  python3 profiles/pmc_summary.py $(find $O/a_$v $O/b_$v $O/c_$v -name '*counter_collection.csv') > $O/summary_$v.txt
done
echo ok
