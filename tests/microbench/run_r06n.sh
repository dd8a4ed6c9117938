#!/bin/bash
# r06n: the round-6 profile set on the current tree: PMC traffic (FETCH_SIZE, WRITE_SIZE) and
# kernel trace + stats per writer job for C2, C3 and C4 (profiles/profile_round.sh), and a C5
# kernel-trace busy / queue summary
set -e
for wl in c2 c3 c4; do
  bash profiles/profile_round.sh r06n $wl > gpurun_out/prof_r06n_$wl.log 2>&1 || { tail -20 gpurun_out/prof_r06n_$wl.log; exit 1; }
  tail -2 gpurun_out/prof_r06n_$wl.log
done
OUT=gpurun_out/r06n_c5
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o run -- python3 bench.py --workload c5 --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --steps 3 --warmup 1 > $OUT/tr.log 2>&1
python3 tests/microbench/trace_busy.py $(find $OUT/tr -name "*kernel_trace.csv" | head -1) 10 > $OUT/busy.txt
python3 tests/microbench/queue_map.py $(find $OUT/tr -name "*kernel_trace.csv" | head -1) > $OUT/queue_map.txt
find $OUT/tr -name "*kernel_trace.csv" -delete
find gpurun_out/prof_r06n_* -name "*kernel_trace.csv" -delete || true
echo done
