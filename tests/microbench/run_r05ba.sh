#!/bin/bash
# r05ba: multi-page metadata read back with the compression's sync, probe headers from the
# min == max flag (no statistics bytes): the multi-page / rotation / parity suites, then the
# per-record legs (128 MiB / 1 MiB / 64 KiB pages) twice
OUT=gpurun_out/r05ba
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multipage.py tests/test_gpu_rotation.py tests/test_gpu_parity.py tests/test_gpu_properties.py > $OUT/tests.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --no-resident --secondary-steps 0 --steps 2 --warmup 1 > $OUT/bench_$r.json 2> $OUT/bench_$r.err || exit $?
done
