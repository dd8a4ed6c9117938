#!/bin/bash
set -e
OUT=gpurun_out/r04e
mkdir -p $OUT
timeout -k 10 300 python -u tests/microbench/diag_c4.py enc 1500000 > $OUT/enc.log 2>&1
timeout -k 10 300 python -u tests/microbench/diag_c4.py writer 1500000 > $OUT/writer.log 2>&1
timeout -k 10 300 python -u tests/microbench/diag_c4.py writer 3000000 >> $OUT/writer.log 2>&1
KPW_EAGER_MB=0 timeout -k 10 300 python -u tests/microbench/diag_c4.py writer 3000000 >> $OUT/writer.log 2>&1
KPW_ENCODERS=1 timeout -k 10 300 python -u tests/microbench/diag_c4.py writer 3000000 >> $OUT/writer.log 2>&1
