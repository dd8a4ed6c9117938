#!/bin/bash
# r05ai: the round's profile set (PMC FETCH/WRITE passes + kernel trace) for c2, c3, c4
set -e
for wl in c2 c3 c4; do
  timeout -k 10 1000 bash profiles/profile_round.sh r05ai $wl > gpurun_out/prof_r05ai_$wl.log 2>&1
done
