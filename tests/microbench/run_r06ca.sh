#!/bin/bash
# per-record loop at 64 KiB pages with spin-wait synchronisation against the default, alternating
for r in 1 2 3; do
  for v in 0 1; do
    echo -n "spin=$v "; PR_SPIN=$v KPW_TRACE=1 timeout -k 10 120 python3 tests/microbench/pr_leg.py 1500000 65536 2>&1 | grep -E "per-record|1293 page" | tr '\n' ' '; echo
  done
done
