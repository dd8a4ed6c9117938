#!/bin/bash
# r04c: diagnose the C4 row-group-1 blob mismatch (seg_bench per-fragment check), a traced C2
# writer run, the default bench line.  From the repo root.
set -e
OUT=gpurun_out/r04c
mkdir -p $OUT
python tests/microbench/dump_rg.py 2 0xC0FFEE04 1500000 1 /tmp/c4rg1.bin > $OUT/dump.log 2>&1
SEG_DUMP_BAD=$OUT/badfrag.bin timeout -k 10 200 tests/microbench/build/seg_bench /tmp/c4rg1.bin 3 > $OUT/seg_c4rg1.log 2>&1 || echo "seg_bench rc=$?" >> $OUT/seg_c4rg1.log
KPW_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/trace_c2.log 2>&1
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1
