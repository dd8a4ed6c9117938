#!/bin/bash
# r05i: k_dict_firsts keeps its count pass's first-occurrence masks for the write pass — parity
# suites, C2/C3 bench lines, C3 kernel trace
OUT=gpurun_out/r05i
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multipage.py tests/test_gpu_rotation.py \
    tests/test_gpu_properties.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0"
for w in c2 c3; do
  for r in 1 2; do
    timeout -k 10 300 $B --workload $w --steps 4 --warmup 1 > $OUT/${w}_$r.json 2> $OUT/${w}_$r.err || exit $?
  done
done
# CUs kept out of the persistent segment kernel's grid (the next job's decode + planning run there)
for rc in 16 32; do
  for w in c2 c3; do
    KPW_SEG_RESERVE_CUS=$rc timeout -k 10 300 $B --workload $w --steps 4 --warmup 1 > $OUT/${w}_rc$rc.json 2> $OUT/${w}_rc$rc.err || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c3 -- $B --workload c3 \
    --steps 2 --warmup 1 > $OUT/c3_prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c2 -- $B --workload c2 \
    --steps 2 --warmup 1 > $OUT/c2_prof.log 2>&1 || exit $?
