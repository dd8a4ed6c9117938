#!/bin/bash
# r06p: the final-tree checks: whole GPU suite and smoke, the profile set (C2 / C3 / C4 PMC
# traffic + kernel stats per writer job), then the driver's bench command
set -e
OUT=gpurun_out/r06p
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
for wl in c2 c3 c4; do
  bash profiles/profile_round.sh r06p $wl > gpurun_out/prof_r06p_$wl.log 2>&1 || { tail -20 gpurun_out/prof_r06p_$wl.log; exit 1; }
done
find gpurun_out/prof_r06p_* -name "*kernel_trace.csv" -delete || true
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
echo done
