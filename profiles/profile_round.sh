#!/bin/bash
# One GPU session of measurements for a round: the default bench line, a rocprofv3 kernel-trace
# --stats run of the same command, and the two PMC passes (FETCH_SIZE, WRITE_SIZE) that
# profiles/collect_traffic.py turns into per-kernel HBM bytes.  Usage: profiles/profile_round.sh OUTDIR [bench args]
set -e
OUT=${1:-gpurun_out/prof}; shift || true
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOTDIR/$OUT"
cd "$ROOTDIR"
timeout -k 10 400 python3 bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
cd /tmp && export TMPDIR=/tmp && cd "$ROOTDIR"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ks" -o run -- python3 bench.py --no-cpu-baseline "$@" > "$OUT/ks.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py --no-cpu-baseline "$@" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py --no-cpu-baseline "$@" > "$OUT/write.log" 2>&1
echo done
