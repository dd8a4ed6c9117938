#!/bin/bash
# Collect the round's profiles of one workload on a GPU box (run from the repo root, e.g.
# through gpurun):
#   profiles/profile_round.sh r03a c2
# Every pass runs bench.py --no-resident --no-cpu-baseline --warmup 0 (every kernel launch belongs
# to a writer encode job of the bench line's timed steps).  1) and 2) separate PMC passes for HBM traffic (FETCH_SIZE and WRITE_SIZE
# do not fit one pass on gfx950), summarised per job into profiles/<tag>_<wl>_pmc_traffic.json;
# 3) the kernel trace + stats pass, whose bench line then reads that file (roofline.traffic);
# 4) the summary.  Every GPU step has its own time limit; the script stops at the first failure.
set -e
TAG=${1:?tag}
WL=${2:-c2}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_${TAG}_${WL}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
ARGS="--workload $WL --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 bench.py $ARGS --steps 3 --warmup 0 > "$OUT/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 bench.py $ARGS --steps 3 --warmup 0 > "$OUT/write.log" 2>&1
python3 profiles/summarize.py pmc "$TAG" "$WL"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py $ARGS --steps 3 --warmup 0 > "$OUT/trace.log" 2>&1
python3 profiles/summarize.py all "$TAG" "$WL"
