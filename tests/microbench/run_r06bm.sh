#!/bin/bash
# bulk multi-page leg: the tree's library against builds at earlier round-6 commits (KPW_GPU_LIB),
# alternating on one box
OUT=gpurun_out/r06bm
mkdir -p $OUT
A="--no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --steps 2 --warmup 1 --secondary-steps 3"
for r in 1 2; do
  for v in tree 55319b4 a2a2a98; do
    if [ $v = tree ]; then L=""; else L="KPW_GPU_LIB=tests/microbench/build/libvar/lib_$v.so"; fi
    env $L KPW_BENCH_LEGS=bulk_multipage timeout -k 10 300 python3 bench.py $A > $OUT/bulk_${v}_$r.json 2> $OUT/bulk_${v}_$r.err || exit 1
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06bm/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    b = d["bulk_multipage"]
    print(f.split("/")[-1], "C2", d["value"], "bulk", b["value"], b["step_ms"], b["writer_phase_ms_mean"], b.get("h2d_gbps"))
PY
