#!/bin/bash
# r04p: the hybrid scans (multi-job and long-run scans back to reduce-then-scan, element tiles
# keep look-back), resident c2/c3/c4 A/B vs the pre-look-back build, traces, the c2 writer line.

OUT=gpurun_out/r04p
mkdir -p $OUT
V=tests/microbench/build/libvar/libkpw_r04pre.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1 || exit $?
for wl in c2 c3 c4; do
  timeout -k 10 200 python3 tests/microbench/resident_only.py $wl > $OUT/res_${wl}_new.log 2>&1 || exit $?
  KPW_GPU_LIB=$V timeout -k 10 200 python3 tests/microbench/resident_only.py $wl > $OUT/res_${wl}_old.log 2>&1 || exit $?
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/w_new_$r.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/res_prof -o run -- python3 tests/microbench/resident_only.py c2 > $OUT/res_prof.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/res_prof3 -o run -- python3 tests/microbench/resident_only.py c3 > $OUT/res_prof3.log 2>&1
