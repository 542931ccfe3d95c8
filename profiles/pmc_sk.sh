#!/bin/bash
# A/B PMC passes of the counting kernels: --superkmer vs --window-records.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/sk}
mkdir -p $O
for mode in "--superkmer" "--window-records"; do
  tag=${mode:-sk}; tag=${tag#--}
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR --output-format csv -d $O/a_$tag -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $mode > $O/a_$tag.log 2>&1
  timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/b_$tag -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $mode > $O/b_$tag.log 2>&1
  timeout -k 10 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/c_$tag -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $mode > $O/c_$tag.log 2>&1
  python3 profiles/pmc_summary.py $O/a_$tag $O/b_$tag $O/c_$tag > $O/summary_$tag.txt
done
echo ok
