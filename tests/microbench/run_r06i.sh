#!/bin/bash
# r06i: pad stream per stream set (queue rotation): C5 queue map and throughput with / without
# pads at 8 and 16 hardware queues; C2 unchanged?; a kernel trace of the 64 KiB per-record loop
OUT=gpurun_out/r06i
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="--workload c5 --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --steps 5 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- python3 bench.py $A > $OUT/tr.log 2>&1 || exit 1
python3 tests/microbench/queue_map.py $(find $OUT/tr -name "*kernel_trace.csv" | head -1) > $OUT/queue_map.txt
find $OUT/tr -name "*kernel_trace.csv" -delete
for r in 1 2; do
  for q in 8 16; do
    for p in 1 0; do
      KPW_STREAM_PAD=$p GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py $A > $OUT/c5_q${q}_p${p}_$r.json 2> $OUT/c5_q${q}_p${p}_$r.err || exit 1
    done
  done
done
B="--no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --steps 10 --warmup 2"
for q in 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py $B > $OUT/c2_q$q.json 2> $OUT/c2_q$q.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/pr -o pr64k -- python3 tests/microbench/pr_leg.py 300000 65536 > $OUT/pr64k.log 2>&1 || exit 1
find $OUT/pr -name "*kernel_trace.csv" -delete
echo done
