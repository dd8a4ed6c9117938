#!/bin/bash
# Test infrastructure: K7 pipeline breakdown at a larger fragment count (8 copies of a C2 row
# group, 2 of the C4 pages), from the repo root through gpurun.
set -e
mkdir -p gpurun_out
python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin
python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin
timeout -k 10 120 tests/microbench/build/seg_bench /tmp/p2.bin 2 8 > gpurun_out/seg2_c2.log 2>&1
timeout -k 10 120 tests/microbench/build/seg_bench /tmp/p4.bin 2 4 > gpurun_out/seg2_c4.log 2>&1
