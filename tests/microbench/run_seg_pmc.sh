#!/bin/bash
# Test infrastructure: K7 segment-kernel phase profile + HBM traffic on a GPU box (through gpurun),
# from the repo root:  tests/microbench/run_seg_pmc.sh TAG
# Dumps C2 / C4 page bodies with the CPU oracle, runs seg_bench (byte identity vs the oracle,
# timings, per-fragment phase cycles), then FETCH_SIZE / WRITE_SIZE passes over the C2 run.
set -e
TAG=${1:-seg}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin
python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin
timeout -k 10 120 tests/microbench/build/seg_bench /tmp/p2.bin 3 > "$OUT/seg_c2.log" 2>&1
timeout -k 10 120 tests/microbench/build/seg_bench /tmp/p4.bin 3 > "$OUT/seg_c4.log" 2>&1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- tests/microbench/build/seg_bench /tmp/p2.bin 1 > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- tests/microbench/build/seg_bench /tmp/p2.bin 1 > "$OUT/write.log" 2>&1
