#!/bin/bash
# Collect the round's profiles on a GPU box (run from the repo root, e.g. through gpurun):
#   profiles/profile_round.sh r01c
# 1) kernel trace + stats of the bench command, 2) and 3) separate PMC passes for HBM
# traffic (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).  Then
#   python profiles/summarize.py r01c   (here or on the box) writes profiles/r01c_*.
set -e
TAG=${1:?tag}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --no-cpu-baseline --steps 3 > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 bench.py --no-cpu-baseline --steps 2 > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 bench.py --no-cpu-baseline --steps 2 > "$OUT/write.log" 2>&1
python3 profiles/summarize.py "$TAG"
