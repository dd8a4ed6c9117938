#!/bin/bash
# SQ counter passes over the Snappy microbench, one rocprofv3 run per pass.
#   tests/microbench/pmc_snappy.sh TAG [snappy_bench args...]   (default args: 96 ts)
set -e
TAG=${1:-ts}
shift || true
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(96 ts)
OUT=gpurun_out/pmc_snappy_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d "$OUT/p1" -o run -- tests/microbench/build/snappy_bench "${ARGS[@]}" > "$OUT/p1.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU --output-format csv -d "$OUT/p2" -o run -- tests/microbench/build/snappy_bench "${ARGS[@]}" > "$OUT/p2.log" 2>&1
