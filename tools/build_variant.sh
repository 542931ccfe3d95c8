#!/bin/bash
# build_variant.sh NAME [extra hipcc flags]: libeulerhip.so variant into exp/lib_NAME.so (experiments)
set -e
NAME=$1; shift
cd "$(dirname "$0")/../pycuda-euler_amd/csrc"
B=/tmp/b_$NAME; mkdir -p $B /root/repo/exp
for f in assemble.hip modules.hip; do /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics "$@" -c -o $B/${f%.hip}.o $f 2>/dev/null & done
for f in capi.cpp ingest.cpp; do /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -x hip -c -o $B/${f%.cpp}.o $f 2>/dev/null & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o /root/repo/exp/lib_$NAME.so $B/*.o
