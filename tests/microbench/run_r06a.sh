#!/bin/bash
# r06a: GPU suite on the round-6 tree (look-back release fence, size_polled, allocator counters),
# then C5 standalone vs in the bench line (allocator calls, per-writer walls, fallbacks), and the
# in-line run with unpooled streams
OUT=gpurun_out/r06a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0"
timeout -k 10 400 $B --workload c5 --secondary-steps 0 --steps 3 --warmup 1 > $OUT/c5_alone.json 2> $OUT/c5_alone.err || exit $?
timeout -k 10 600 $B --steps 5 --warmup 1 > $OUT/line.json 2> $OUT/line.err || exit $?
KPW_STREAM_POOL=0 timeout -k 10 600 $B --steps 5 --warmup 1 > $OUT/line_nopool.json 2> $OUT/line_nopool.err || exit $?
KPW_TRACE=1 timeout -k 10 400 $B --workload c5 --secondary-steps 0 --steps 2 --warmup 1 > $OUT/c5_alone_tr.json 2> $OUT/c5_alone_tr.err || exit $?
echo done
