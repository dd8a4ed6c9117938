#!/bin/bash
# Test infrastructure: kernel + memory-copy + HIP API trace of one C3 writer step (which host
# calls produce the __amd_rocclr_copyBuffer / fillBuffer blit kernels), summarised on the box
# (the raw CSVs exceed what gpurun copies back).  No counters in this pass.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W=${1:-c3}
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d /tmp/ctr -o run -- \
    python3 bench.py --workload $W --no-cpu-baseline --no-resident --steps 1 --warmup 0 > gpurun_out/${W}trace.log 2>&1
python3 tests/microbench/trace_copies.py /tmp/ctr > gpurun_out/${W}trace_summary.txt 2>&1
