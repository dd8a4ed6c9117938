#!/bin/bash
# Test infrastructure: builds tests/microbench/build/seg_bench (working tree) plus -D variants
# given as name=flags arguments, and seg_bench_base from git HEAD's k_snappy_seg.hip when
# BASE=1.  Run from tests/microbench.
set -e
F="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I../../include -mllvm -sink-insts-to-avoid-spills"
mkdir -p build
gcc -O2 -c ../../oracle/oracle_snappy.c -I../../include -o build/oracle_snappy.o
one() {   # name srcdir flags
  /opt/rocm/bin/hipcc $F -I$2/kafka-parquet-writer_amd/csrc $3 -c $2/tests/microbench/seg_bench.hip -o build/$1.o 2>/dev/null
  /opt/rocm/bin/hipcc --offload-arch=gfx950 build/$1.o build/oracle_snappy.o -o build/$1
  rm -f build/$1.o
}
if [ "$BASE" = 1 ]; then
  B=/tmp/seg_basesrc; rm -rf $B; mkdir -p $B/kafka-parquet-writer_amd/csrc $B/tests/microbench
  cp ../../kafka-parquet-writer_amd/csrc/*.h ../../kafka-parquet-writer_amd/csrc/k_snappy.hip $B/kafka-parquet-writer_amd/csrc/
  (cd ../.. && git show HEAD:kafka-parquet-writer_amd/csrc/k_snappy_seg.hip) > $B/kafka-parquet-writer_amd/csrc/k_snappy_seg.hip
  cp seg_bench.hip $B/tests/microbench/
  one seg_bench_base $B "" &
fi
R=$(cd ../.. && pwd)
one seg_bench $R "" &
for a in "$@"; do one seg_bench_${a%%=*} $R "${a#*=}" & done
wait
ls build
