set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/g13; mkdir -p $O
for v in 0 1; do
EULERHIP_PACK12=$v timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $O/a$v -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/a$v.log 2>&1 || exit 1
EULERHIP_PACK12=$v timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE TCP_TCC_READ_REQ_sum --output-format csv -d $O/b$v -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/b$v.log 2>&1 || exit 1
python3 profiles/pmc_summary.py $O/a$v $O/b$v > $O/summary$v.txt
done
grep -A12 "^k_bucket$" $O/summary0.txt $O/summary1.txt
