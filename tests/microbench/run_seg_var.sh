#!/bin/bash
# Test infrastructure: runs every tests/microbench/build/seg_bench_* variant (built on the CPU
# side with different -D settings) on the C2 and C4 page dumps; one log per variant and workload.
set -e
mkdir -p gpurun_out
python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin
python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin
for b in tests/microbench/build/seg_bench_*; do
    v=$(basename $b)
    timeout -k 10 120 $b /tmp/p2.bin 3 > gpurun_out/${v}_c2.log 2>&1
    timeout -k 10 120 $b /tmp/p4.bin 3 > gpurun_out/${v}_c4.log 2>&1
done
if [ -n "$SEG_C3" ]; then
    python tests/microbench/dump_any.py 3 400000 /tmp/p3.bin
    for b in tests/microbench/build/seg_bench_*; do
        v=$(basename $b)
        timeout -k 10 120 $b /tmp/p3.bin 3 > gpurun_out/${v}_c3.log 2>&1
    done
fi
