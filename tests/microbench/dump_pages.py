"""Test-infrastructure helper: encode N Rec8 records with the CPU oracle (UNCOMPRESSED, bench
properties) and dump every page body as (u64 length, bytes) records for snappy_stats.
  python tests/microbench/dump_pages.py 2200000 /tmp/pages.bin"""
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


def main():
    n, path = int(sys.argv[1]), sys.argv[2]
    d, o = synth.generate(synth.KIND_REC8, 1, n)
    props = oracle.make_props(block_size=128 * MiB, page_size=128 * MiB, codec=0, enable_dictionary=True)
    fb = oracle.encode_file(synth.REC8, d, o, props)
    with open(path, "wb") as f:
        for pg in pqwalk.pages(fb):
            if pg["rg"] != 0:
                continue
            f.write(struct.pack("<Q", len(pg["body"])))
            f.write(pg["body"])
            print(pg["col"], pg["header"][1], len(pg["body"]))


if __name__ == "__main__":
    main()
