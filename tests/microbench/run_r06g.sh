#!/bin/bash
# r06g: probe dictionary continuation (rotation + multi-page parity, per-record legs), then C5
# after each other secondary leg (which leg leaves the process slower for C5)
OUT=gpurun_out/r06g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_rotation.py tests/test_gpu_multipage.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
A="--no-cpu-baseline --no-resident --steps 5 --warmup 1"
timeout -k 10 600 python3 bench.py $A --per-record-records 1000000 > $OUT/pr.json 2> $OUT/pr.err || exit 1
KPW_PROBE_CONT=0 timeout -k 10 600 python3 bench.py $A --per-record-records 1000000 --secondary-steps 0 > $OUT/pr_nocont.json 2> $OUT/pr_nocont.err || exit 1
for o in "c5" "c4,c5" "bulk_multipage,c5" "c3,c5" "gzip,c5"; do
  KPW_BENCH_LEGS=$o timeout -k 10 600 python3 bench.py $A --per-record-records 0 --per-record-64k-records 0 > "$OUT/legs_$o.json" 2> "$OUT/legs_$o.err" || exit 1
done
echo done
