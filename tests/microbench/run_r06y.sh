#!/bin/bash
# C3 / C2 writer line against the stage-flush bound (KPW_STAGE_FLUSH_MB: the largest fill a
# busy pipeline lets grow before it submits; the last fill is close()'s tail)
set -e
mkdir -p gpurun_out/r06y
A="--no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0"
for rep in 1 2; do
  for mb in 1024 512 768; do
    KPW_STAGE_FLUSH_MB=$mb timeout -k 10 300 python bench.py --workload c3 --steps 5 --warmup 2 $A > gpurun_out/r06y/c3_${mb}_$rep.json 2> gpurun_out/r06y/c3_${mb}_$rep.err
  done
done
for mb in 1024 512; do
  KPW_STAGE_FLUSH_MB=$mb timeout -k 10 300 python bench.py --workload c2 --steps 10 --warmup 3 $A > gpurun_out/r06y/c2_${mb}.json 2> gpurun_out/r06y/c2_${mb}.err
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06y/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d.get("writer_phase_ms_per_step"), d.get("encode_jobs_per_step"))
PY
