#!/bin/bash
# Lab library: the in-tree objects with gemm.hip / gemm_x6p.hip rebuilt under extra defines.
# usage: [LAB_SRCS="a.hip b.hip"] scripts/lab/lab_build.sh OUT.so -DFLAG [-DFLAG ...]
# (run after python -m k3m_amd.build_lib; LAB_SRCS defaults to the two GEMM sources)
set -e
cd "$(dirname "$0")/../.."
out=$1; shift
tmp=$(mktemp -d)
FL="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -mcode-object-version=5 -Wno-unused-result -fno-slp-vectorize"
for s in ${LAB_SRCS:-gemm.hip gemm_x6p.hip}; do /opt/rocm/bin/hipcc $FL "$@" -c k3m_amd/csrc/$s -o $tmp/$s.o & done
wait
objs=""
for o in k3m_amd/build/*.o; do b=$(basename $o); if [ -f $tmp/$b ]; then objs="$objs $tmp/$b"; else objs="$objs $o"; fi; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out" $objs
rm -rf $tmp
echo "$out"
