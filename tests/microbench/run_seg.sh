#!/bin/bash
# Test infrastructure: K7 segment-kernel check on a GPU box (through gpurun), from the repo root:
#   tests/microbench/run_seg.sh [full]
# dumps C2/C4 page bodies with the CPU oracle, runs seg_bench (byte identity vs the oracle +
# timings); "full" also runs the -m gpu suite and the default bench.  Every GPU step has its own
# time limit and the script stops at the first failure.
set -e
mkdir -p gpurun_out
rm -f gpurun_out/seg_c2.log gpurun_out/seg_c4.log gpurun_out/gpu_tests.log gpurun_out/bench_c2.log
python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin
python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin
timeout -k 10 120 tests/microbench/build/seg_bench /tmp/p2.bin 3 > gpurun_out/seg_c2.log 2>&1
timeout -k 10 120 tests/microbench/build/seg_bench /tmp/p4.bin 3 > gpurun_out/seg_c4.log 2>&1
if [ "$1" = full ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
    timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1
fi
