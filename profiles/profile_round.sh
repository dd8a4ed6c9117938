#!/bin/bash
# Collect the round's profiles of one workload on a GPU box (run from the repo root, e.g.
# through gpurun):
#   profiles/profile_round.sh r02a c2
# 1) kernel trace + stats of the bench command, 2) and 3) separate PMC passes for HBM traffic
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).  Every GPU step has its own time
# limit; the script stops at the first failure.  Then
#   python profiles/summarize.py r02a c2   (here or on the box) writes profiles/r02a_c2_*.
set -e
TAG=${1:?tag}
WL=${2:-c2}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_${TAG}_${WL}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
ARGS="--workload $WL --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py $ARGS --steps 3 --warmup 1 > "$OUT/trace.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 bench.py $ARGS --steps 2 --warmup 1 > "$OUT/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 bench.py $ARGS --steps 2 --warmup 1 > "$OUT/write.log" 2>&1
python3 profiles/summarize.py "$TAG" "$WL"
