#!/bin/bash
# r06c: kernel traces of C5 (8 writers) and C2 (one writer) for the GPU busy profile
# (tests/microbench/trace_busy.py), and C4 with 0 / 16 CUs kept out of the segment kernel's
# grid (the other worker's short kernels), alternated twice
OUT=gpurun_out/r06c
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="--no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/c5 -o run -- python3 bench.py --workload c5 $A --steps 2 --warmup 1 > $OUT/c5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/c2 -o run -- python3 bench.py --workload c2 $A --steps 2 --warmup 1 > $OUT/c2.log 2>&1 || exit $?
python3 tests/microbench/trace_busy.py $(find $OUT/c5 -name "*kernel_trace.csv" | head -1) 10 > $OUT/c5_busy.txt
python3 tests/microbench/trace_busy.py $(find $OUT/c2 -name "*kernel_trace.csv" | head -1) 10 > $OUT/c2_busy.txt
for r in 1 2; do
  for rc in 0 16; do
    KPW_SEG_RESERVE_CUS=$rc timeout -k 10 300 python3 bench.py --workload c4 $A --steps 3 --warmup 1 > $OUT/c4_rc${rc}_$r.json 2> $OUT/c4_rc${rc}_$r.err || exit $?
  done
done
find $OUT -name "*kernel_trace.csv" -delete
echo done
