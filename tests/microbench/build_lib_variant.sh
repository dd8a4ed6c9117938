#!/bin/bash
# Test infrastructure: tests/microbench/build/libvar/libkpw_<name>.so = the in-tree objects
# (make first) with the listed sources recompiled under extra flags, for A/B runs through
# KPW_GPU_LIB.  Usage: build_lib_variant.sh <name> "<flags>" src1.hip src2.cpp ...
set -e
name=$1; flags=$2; shift 2
R=$(cd "$(dirname "$0")/../.." && pwd)
P=$R/kafka-parquet-writer_amd
O=/tmp/libvar_$name; rm -rf $O; mkdir -p $O $R/tests/microbench/build/libvar
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-variable -ffp-contract=off"
make -s -C $P
cp $P/build/*.o $O/
for src in "$@"; do
  b=$(basename ${src%.*})
  /opt/rocm/bin/hipcc $F $flags -c $P/csrc/$src -o $O/$b.o &
done
wait
/opt/rocm/bin/hipcc $F -shared -pthread -o $R/tests/microbench/build/libvar/libkpw_$name.so $O/*.o
echo built libkpw_$name.so
