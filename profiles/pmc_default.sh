#!/bin/bash
# SQ PMC passes (three runs: the hardware cannot collect them in one) of the default headline
# bench, summarised per kernel by profiles/pmc_summary.py.  Usage: profiles/pmc_default.sh OUTDIR
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/pmc}
mkdir -p $O
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR --output-format csv -d $O/a -o run -- python3 bench.py --no-cpu-baseline --no-host-input --steps 2 --warmup 1 > $O/a.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/b -o run -- python3 bench.py --no-cpu-baseline --no-host-input --steps 2 --warmup 1 > $O/b.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/c -o run -- python3 bench.py --no-cpu-baseline --no-host-input --steps 2 --warmup 1 > $O/c.log 2>&1
python3 profiles/pmc_summary.py $O/a $O/b $O/c > $O/summary.txt
echo ok
