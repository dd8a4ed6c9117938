#!/bin/bash
# Test infrastructure: FETCH_SIZE / WRITE_SIZE of k_snappy_seg per dispatch for the seg_bench
# variants given as arguments (tests/microbench/build/seg_bench*), on dumped C4 (and C2) pages.
#   tests/microbench/run_seg_attr.sh TAG variant...
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin
python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in "$@"; do
  for k in 4 2; do
    timeout -k 10 120 tests/microbench/build/$v /tmp/p$k.bin 3 > "$OUT/${v}_c$k.log" 2>&1
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/${v}_c${k}_$c" -o run -- tests/microbench/build/$v /tmp/p$k.bin 1 > "$OUT/${v}_c${k}_$c.log" 2>&1
    done
  done
done
