"""Test-infrastructure helper: encode records of one synth kind with the CPU oracle (UNCOMPRESSED)
and dump the page bodies of row group 0 as (u64 length, bytes) records (seg_bench input).
  python tests/microbench/dump_any.py KIND NRECORDS OUT [SEED [BLOCK [PAGE [PARAM]]]]
  KIND 0 SampleMessage, 1 Rec8, 2 HighCard, 3 Wide; BLOCK/PAGE in bytes (default 128 MiB)"""
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("", "tests", "synth", "kafka-parquet-writer_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import oracle  # noqa: E402
import pqwalk  # noqa: E402
import synth  # noqa: E402

MiB = 1024 * 1024
kind, n, path = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
seed = int(sys.argv[4], 0) if len(sys.argv) > 4 else 7
block = int(sys.argv[5]) if len(sys.argv) > 5 else 128 * MiB
page = int(sys.argv[6]) if len(sys.argv) > 6 else 128 * MiB
param = int(sys.argv[7]) if len(sys.argv) > 7 else 0
d, o = synth.generate(kind, seed, n, param=param)
props = oracle.make_props(block_size=block, page_size=page, codec=0, enable_dictionary=True)
fb = oracle.encode_file(synth.SCHEMAS[kind], d, o, props)
with open(path, "wb") as f:
    for pg in pqwalk.pages(fb):
        if pg["rg"] != 0:
            continue
        f.write(struct.pack("<Q", len(pg["body"])))
        f.write(pg["body"])
