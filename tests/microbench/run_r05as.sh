#!/bin/bash
# r05as: the bench line's later legs (c4, gzip) after the per-record legs: default, multi-page round
# growth off, stream pool off
OUT=gpurun_out/r05as
mkdir -p $OUT
B="python bench.py --no-cpu-baseline --no-resident --steps 2 --warmup 1"
timeout -k 10 600 $B > $OUT/def.json 2> $OUT/def.err || exit $?
KPW_MP_ROUND_GROW=1 timeout -k 10 600 $B > $OUT/g1.json 2> $OUT/g1.err || exit $?
KPW_STREAM_POOL=0 timeout -k 10 600 $B > $OUT/np.json 2> $OUT/np.err || exit $?
