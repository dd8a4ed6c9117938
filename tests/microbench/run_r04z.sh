#!/bin/bash
# r04z: fewer dispatches per job (fills folded into kernels, merged uploads, one planner
# prefix scan): GPU suite, resident c2/c3, c2 writer trace.
OUT=gpurun_out/r04z
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1 || exit $?
for wl in c3 c2; do
  timeout -k 10 200 python3 tests/microbench/resident_only.py $wl > $OUT/res_${wl}.log 2>&1 || exit $?
done
for r in 1 2; do timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/w_c2_$r.log 2>&1 || exit $?; done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/w_prof -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/w_prof.log 2>&1
