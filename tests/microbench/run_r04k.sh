#!/bin/bash
# r04k: the round's profiles (kernel trace + FETCH/WRITE PMC passes) of c2, c4, c3 on the
# current build, then the default bench line (which reads the newest traffic files).
set -e
timeout -k 10 600 profiles/profile_round.sh r04c c2
timeout -k 10 600 profiles/profile_round.sh r04c c4
timeout -k 10 600 profiles/profile_round.sh r04c c3
timeout -k 10 600 python bench.py > gpurun_out/r04c_bench.log 2>&1
