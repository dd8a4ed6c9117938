"""Test-infrastructure helper: the page bodies (UNCOMPRESSED, CPU oracle) of one row group of a
synth workload's record stream, as seg_bench input ((u64 length, bytes) records).
  python tests/microbench/dump_rg.py KIND SEED NRECORDS RG OUT [COL]
NRECORDS must cover row group RG (+ 10001 records); COL limits the dump to one column."""
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("", "tests", "synth", "kafka-parquet-writer_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import oracle  # noqa: E402
import pqwalk  # noqa: E402
import synth  # noqa: E402

kind, seed, n, rg, path = int(sys.argv[1]), int(sys.argv[2], 0), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
col = int(sys.argv[6]) if len(sys.argv) > 6 else -1
d, o = synth.generate(kind, seed, n)
fb = oracle.encode_file(synth.SCHEMAS[kind], d, o, oracle.make_props(codec=0))
nrg = len(pqwalk.footer(fb)[4])
assert rg < nrg - 1, "NRECORDS does not cover row group %d (%d row groups)" % (rg, nrg)
with open(path, "wb") as f:
    for pg in pqwalk.pages(fb):
        if pg["rg"] != rg or (col >= 0 and pg["col"] != col):
            continue
        print("rg %d col %d page type %d len %d" % (pg["rg"], pg["col"], pg["header"][1], len(pg["body"])))
        f.write(struct.pack("<Q", len(pg["body"])))
        f.write(pg["body"])
