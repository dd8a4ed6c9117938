#!/bin/bash
# Test infrastructure: which copy engine serves the writer's H2D (env + a short bench each way).
mkdir -p gpurun_out
env | grep -iE "sdma|blit|HSA_|GPU_MAX" > gpurun_out/sdma_env.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/sdma_default.log 2>&1 || exit 1
HSA_ENABLE_SDMA=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/sdma_on.log 2>&1 || exit 1
HSA_ENABLE_SDMA=0 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/sdma_off.log 2>&1 || exit 1
