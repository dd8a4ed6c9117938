#!/bin/bash
# r05h: small copies without CUs.  nocu_probe (does a 1 KiB copy wait for a kernel holding every
# CU?), parity with KPW_SMALL_NOCU=1, then C2/C3 A/B (default blit copies vs KPW_SMALL_NOCU=1)
OUT=gpurun_out/r05h
mkdir -p $OUT
timeout -k 10 60 tests/microbench/build/nocu_probe > $OUT/probe.log 2>&1 || exit $?
KPW_SMALL_NOCU=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multipage.py -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest_nocu.log 2>&1 || exit $?
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0"
for w in c2 c3; do
  for r in 1 2; do
    timeout -k 10 300 $B --workload $w --steps 4 --warmup 1 > $OUT/${w}_a$r.json 2> $OUT/${w}_a$r.err || exit $?
    KPW_SMALL_NOCU=1 timeout -k 10 300 $B --workload $w --steps 4 --warmup 1 > $OUT/${w}_n$r.json 2> $OUT/${w}_n$r.err || exit $?
  done
done
