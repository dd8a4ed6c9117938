set -e
for r in 0 32 64; do
  for wl in c2 c4; do
    KPW_SEG_RESERVE_CUS=$r timeout -k 10 300 python bench.py --workload $wl --steps 6 --warmup 2 --no-cpu-baseline --per-record-records 0 > gpurun_out/resv_${r}_${wl}.log 2>&1
  done
done
