#!/bin/bash
# r05aj: single-page dictionary insertion in two launches (KPW_DICT_SPLIT_TILES 256 / 0) and the
# block-parallel k_mp_satisfy — parity suites, then C2 / C3 / C4 lines alternating
OUT=gpurun_out/r05aj
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_multipage.py tests/test_gpu_rotation.py tests/test_gpu_wire.py > $OUT/pytest.log 2>&1 || exit $?
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --steps 4 --warmup 1"
for r in 1 2; do
  for sp in 0 256; do
    for w in c2 c4; do
      KPW_DICT_SPLIT_TILES=$sp timeout -k 10 300 $B --workload $w > $OUT/${w}_s${sp}_$r.json 2> $OUT/${w}_s${sp}_$r.err || exit $?
    done
  done
done
timeout -k 10 300 $B --workload c3 > $OUT/c3_s256.json 2> $OUT/c3_s256.err || exit $?
KPW_DICT_SPLIT_TILES=0 timeout -k 10 300 $B --workload c3 > $OUT/c3_s0.json 2> $OUT/c3_s0.err || exit $?
