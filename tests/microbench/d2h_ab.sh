#!/bin/bash
# Test infrastructure: writer bench A/B, one D2H per job (default) vs per-page D2H into the arena.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 > gpurun_out/d2h_job.log 2>&1
KPW_D2H_PER_PAGE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 > gpurun_out/d2h_page.log 2>&1
