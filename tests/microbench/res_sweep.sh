#!/bin/bash
# Test infrastructure: resident-only encodes (tests/microbench/resident_only.py) under several
# environment settings, kernel-traced: ENV_CFGS="tag:VAR=1;tag2:VAR=2" WL=c2
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
IFS=';' read -ra CFGS <<< "${ENV_CFGS:?}"
for cfg in "${CFGS[@]}"; do
  tag=${cfg%%:*}; vars=${cfg#*:}
  ( export $vars; timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/res_${tag} -o run -- python3 tests/microbench/resident_only.py ${WL:-c2} > gpurun_out/res_${tag}.log 2>&1 )
done
