#!/bin/bash
# r04u: planner events per group of 8 positions (E8): GPU suite (minus full size), resident
# c2/c3 with kernel traces, the c2 writer line.
OUT=gpurun_out/r04u
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1 || exit $?
for wl in c2 c3; do
  timeout -k 10 200 python3 tests/microbench/resident_only.py $wl > $OUT/res_${wl}.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/w.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/res_prof3 -o run -- python3 tests/microbench/resident_only.py c3 > $OUT/res_prof3.log 2>&1
