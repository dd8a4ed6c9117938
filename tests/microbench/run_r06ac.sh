#!/bin/bash
# C2 writer line against the eager job size (KPW_EAGER_MB) on the round-6 pipeline, alternating
set -e
mkdir -p gpurun_out/${OUT:-r06ac}
A="--no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0"
for rep in 1 2; do
  for mb in ${MBS:-384 256 320 448}; do
    KPW_EAGER_MB=$mb timeout -k 10 300 python bench.py --workload c2 --steps 10 --warmup 3 $A > gpurun_out/${OUT:-r06ac}/c2_${mb}_$rep.json 2> gpurun_out/${OUT:-r06ac}/c2_${mb}_$rep.err
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/${OUT:-r06ac}/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d.get("writer_phase_ms_per_step"), d.get("encode_jobs_per_step"), d.get("h2d_gbps"))
PY
