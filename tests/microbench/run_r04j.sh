#!/bin/bash
# r04j: full-size / multi-page / per-record GPU tests on the current build, the bulk multi-page
# leg under KPW_TRACE and rocprofv3, the per-record legs, and the K7 seg bench of this build.
OUT=gpurun_out/r04j
mkdir -p $OUT
python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin > /dev/null
python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin > /dev/null
for k in 2 4; do timeout -k 10 120 tests/microbench/build/seg_bench /tmp/p$k.bin 3 > $OUT/seg_c$k.log 2>&1 || exit $?; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread -k "fullsize or reference_defaults or every_record" > $OUT/pytest.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/mp_leg.py 10000000 1048576 3 > $OUT/mp_trace.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 1 --warmup 0 --no-resident --no-cpu-baseline --secondary-steps 0 --per-record-records 3000000 > $OUT/per_record.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mp_prof -o run -- python tests/microbench/mp_leg.py 10000000 1048576 2 > $OUT/mp_prof.log 2>&1
