#!/bin/bash
# r05c: k_snappy_seg in quota mode (workgroups of q fragments with pooled scratch instead of the
# persistent grid) and K7 on a low-priority stream: parity first, then the C2 step / close tail
# and C4 per setting
OUT=gpurun_out/r05c
mkdir -p $OUT
KPW_SEG_QUOTA=1 KPW_K7_LOWPRI=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "snappy_patterns or pages_match_oracle or writer_file_identical or eager" \
    -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
KPW_SEG_QUOTA=2 KPW_K7_LOWPRI=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k "c4" \
    -x -q --timeout 200 --timeout-method thread >> $OUT/pytest.log 2>&1 || exit $?
A="--no-resident --no-cpu-baseline --per-record-records 0 --secondary-steps 0 --steps 4 --warmup 1"
for cfg in "0 0" "1 0" "2 0" "4 0" "0 1" "2 1"; do
  set -- $cfg
  KPW_TRACE=1 KPW_SEG_QUOTA=$1 KPW_K7_LOWPRI=$2 timeout -k 10 120 python bench.py $A > $OUT/c2_q$1_p$2.log 2>&1 || exit $?
  KPW_SEG_QUOTA=$1 KPW_K7_LOWPRI=$2 timeout -k 10 120 python bench.py $A --workload c4 --steps 2 > $OUT/c4_q$1_p$2.log 2>&1 || exit $?
done
