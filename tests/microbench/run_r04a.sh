#!/bin/bash
# r04a: seg kernel A/B (staged scatter) + traffic, the GPU suite, a traced C2 writer run, the
# default bench line.  From the repo root through gpurun.
set -e
OUT=gpurun_out/r04a
mkdir -p $OUT
python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin
python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin
for v in seg_bench seg_bench_stg; do
  for k in 2 4; do
    timeout -k 10 120 tests/microbench/build/$v /tmp/p$k.bin 3 > $OUT/${v}_c$k.log 2>&1
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/stg_c4_$c -o run -- tests/microbench/build/seg_bench_stg /tmp/p4.bin 1 > $OUT/stg_c4_$c.log 2>&1
done
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
KPW_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/trace_c2.log 2>&1
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1
