#!/bin/bash
# r06o: look-back publish ordered by waiting for the status store (no L2 write-back): look-back
# and parity tests, then kernel traces of C2 and C3 (k_phase / k_r_sizes against r05 / r06n),
# and the C2 / C3 lines
OUT=gpurun_out/r06o
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_lookback.py tests/test_gpu_parity.py tests/test_gpu_multipage.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="--no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0"
for wl in c2 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_$wl -o run -- python3 bench.py --workload $wl $A --steps 3 --warmup 0 > $OUT/tr_$wl.log 2>&1 || exit 1
  find $OUT/tr_$wl -name "*kernel_trace.csv" -delete
done
timeout -k 10 300 python3 bench.py --workload c3 $A --steps 4 --warmup 1 > $OUT/c3.json 2> $OUT/c3.err || exit 1
timeout -k 10 300 python3 bench.py --workload c2 $A --steps 8 --warmup 2 > $OUT/c2.json 2> $OUT/c2.err || exit 1
echo done
