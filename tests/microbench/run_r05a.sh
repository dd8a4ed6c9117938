#!/bin/bash
# r05a: the round-5 additions on the GPU (C5 at its stated shape, async-batch release by every
# entry point), then the default bench line (now with its c5 key)
OUT=gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py::test_c5_concurrent_writers_full_size \
    tests/test_gpu_async_write.py tests/test_gpu_concurrent.py -x -v --timeout 500 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 500 python bench.py > $OUT/bench.log 2>&1 || exit $?
