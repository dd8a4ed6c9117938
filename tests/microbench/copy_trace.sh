#!/bin/bash
# Test infrastructure: kernel + memory-copy trace of a short writer bench (which copies are SDMA,
# which run as blit kernels).  No counters in this pass.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/ctrace -o run -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/ctrace.log 2>&1
