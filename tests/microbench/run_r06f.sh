#!/bin/bash
# r06f: probes that encode only the newly cut pages (rotation + multi-page parity), then the C5
# leg first vs last in the bench line with the GPU's clocks / power / temperature sampled
OUT=gpurun_out/r06f
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_rotation.py tests/test_gpu_multipage.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
( for i in $(seq 1 400); do echo "T $SECONDS"; rocm-smi -c -P -t --csv 2>/dev/null | grep -v "^$" | tail -n +2; sleep 0.5; done ) > $OUT/smi.log 2>&1 &
SMI=$!
A="--no-cpu-baseline --no-resident --per-record-records 0"
echo "first start $SECONDS" > $OUT/marks.txt
KPW_BENCH_C5_FIRST=1 timeout -k 10 600 python3 bench.py $A --steps 20 --warmup 5 > $OUT/c5first.json 2> $OUT/c5first.err || { kill $SMI; exit 1; }
echo "last start $SECONDS" >> $OUT/marks.txt
timeout -k 10 600 python3 bench.py $A --steps 20 --warmup 5 > $OUT/c5last.json 2> $OUT/c5last.err || { kill $SMI; exit 1; }
echo "end $SECONDS" >> $OUT/marks.txt
kill $SMI
echo done
