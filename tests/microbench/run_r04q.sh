#!/bin/bash
# r04q: packed host tables (one upload per stage), one page-table readback per phase, the
# self-resetting K7 fragment counter: GPU suite (minus full size), seg bench, resident c2/c3,
# the c2 writer line x2, and a kernel trace of the c2 writer (dispatches per job).
OUT=gpurun_out/r04q
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1 || exit $?
python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin > /dev/null
timeout -k 10 120 tests/microbench/build/seg_bench /tmp/p2.bin 3 > $OUT/seg_c2.log 2>&1 || exit $?
for wl in c2 c3; do
  timeout -k 10 200 python3 tests/microbench/resident_only.py $wl > $OUT/res_${wl}.log 2>&1 || exit $?
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/w_$r.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/w_prof -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/w_prof.log 2>&1
