#!/bin/bash
# r05d: (1) kernel + memory-copy + HIP API trace of one C3 writer step, summarised on the box
# (which host calls produce the __amd_rocclr_copyBuffer blits, their sizes and durations);
# (2) seg_bench phase counters on dumped C2 / C3 / C4 pages (K7 baseline for this round)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05d
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d /tmp/ctr -o run -- \
    python3 bench.py --workload c3 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 --steps 1 --warmup 0 > $OUT/c3trace.log 2>&1
python3 tests/microbench/trace_copies.py /tmp/ctr > $OUT/c3trace_summary.txt 2>&1
test -x tests/microbench/build/seg_bench
python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin
python tests/microbench/dump_any.py 3 100000 /tmp/p3.bin
python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin
for k in 2 3 4; do
  timeout -k 10 120 tests/microbench/build/seg_bench /tmp/p$k.bin 3 > $OUT/seg_c$k.log 2>&1
done
