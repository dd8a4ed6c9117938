#!/bin/bash
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 tests/microbench/build/h2d_probe > gpurun_out/h2d.log 2>&1
timeout -k 10 100 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/h2dprof -o run -- tests/microbench/build/h2d_probe > gpurun_out/h2d_prof.log 2>&1
