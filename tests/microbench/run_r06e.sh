#!/bin/bash
# r06e: the driver's bench command on the round-6 tree (caches trimmed between legs, C5 with two
# warm-up steps, dynamic device cache cap), timed
OUT=gpurun_out/r06e
mkdir -p $OUT
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "wall $SECONDS s"; [ $rc -eq 0 ] || exit $rc
# || exit $?
echo done
