#!/bin/bash
# r05g: long-run tiles of 16384 positions (64-bit break masks per thread) — parity suites; C3 and
# C2 bench lines with the file-bytes D2H as a blit kernel (default) and as a no-CU copy (SDMA)
OUT=gpurun_out/r05g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multipage.py tests/test_gpu_wire.py \
    tests/test_gpu_properties.py tests/test_gpu_rotation.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0"
for w in c3 c2; do
  timeout -k 10 300 $B --workload $w --steps 4 --warmup 1 > $OUT/${w}_a.json 2> $OUT/${w}_a.err || exit $?
  KPW_ASM_NOCU=1 timeout -k 10 300 $B --workload $w --steps 4 --warmup 1 > $OUT/${w}_nocu.json 2> $OUT/${w}_nocu.err || exit $?
  timeout -k 10 300 $B --workload $w --steps 4 --warmup 1 > $OUT/${w}_a2.json 2> $OUT/${w}_a2.err || exit $?
  KPW_ASM_NOCU=1 timeout -k 10 300 $B --workload $w --steps 4 --warmup 1 > $OUT/${w}_nocu2.json 2> $OUT/${w}_nocu2.err || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c3 -- $B --workload c3 \
    --steps 2 --warmup 1 > $OUT/c3_prof.log 2>&1 || exit $?
