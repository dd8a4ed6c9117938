#!/bin/bash
# r05f: tile maps + dictionary order expanded on the device (k_maps.hip): parity suites, then C3
# (bench line + copy trace + kernel stats)
OUT=gpurun_out/r05f
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multipage.py tests/test_gpu_wire.py -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline --steps 3 --warmup 1 > $OUT/c3_bench.json 2> $OUT/c3_bench.err || exit $?
KPW_COPY_TRACE=1 timeout -k 10 200 python bench.py --workload c3 --no-cpu-baseline --no-resident \
    --per-record-records 0 --secondary-steps 0 --steps 1 --warmup 1 > $OUT/c3_copies.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c3 -- python bench.py --workload c3 --no-cpu-baseline \
    --no-resident --per-record-records 0 --secondary-steps 0 --steps 2 --warmup 1 > $OUT/c3_prof.log 2>&1 || exit $?
