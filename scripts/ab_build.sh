#!/bin/bash
# usage: ab_build.sh <name> <extra flags...>: rebuild the re-rank / coarse TUs with the flags, link a variant lib
set -e
name=$1; shift
cd /root/repo/hnsw-ivf_amd
out=/tmp/ab_$name; mkdir -p $out
FL="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result -Wno-unused-variable -Wno-sign-compare -Wno-unused-value --offload-arch=gfx950"
VAR=${VAR:-"kernels_ivf_rerank kernels_ivfpq_rerank_d2 kernels_ivfpq_rerank_d4 kernels_ivfpq_rerank_d8 kernels_coarse"}
for f in $VAR; do /opt/rocm/bin/hipcc $FL "$@" -c csrc/$f.hip -o $out/$f.o & done
wait
objs=""
for o in build/*.o; do b=$(basename $o .o); if echo " $VAR " | grep -q " $b "; then objs="$objs $out/$b.o"; else objs="$objs $o"; fi; done
mkdir -p lib/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/ab/libfaiss_amd_$name.so $objs -Wl,-soname,libfaiss_amd.so -lpthread -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built lib/ab/libfaiss_amd_$name.so
