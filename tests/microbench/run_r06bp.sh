#!/bin/bash
# c5 and c4 legs: the tree's library against the build at 55319b4, alternating on one box
OUT=gpurun_out/r06bp
mkdir -p $OUT
A="--no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --steps 2 --warmup 1"
for r in 1 2; do
  for v in tree 55319b4; do
    if [ $v = tree ]; then L=""; else L="KPW_GPU_LIB=tests/microbench/build/libvar/lib_$v.so"; fi
    env $L KPW_BENCH_LEGS=c5,c4 timeout -k 10 400 python3 bench.py $A > $OUT/l_${v}_$r.json 2> $OUT/l_${v}_$r.err || exit 1
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06bp/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], "C2", d["value"], "c5", d["c5"]["value"], d["c5"]["step_ms"], "c4", d["c4"]["value"])
PY
