"""Test infrastructure: a GZIP writer line (C2 Rec8 records, 128 MiB row groups and pages, bulk
writes through ParquetFile), for timing K7' (k_deflate.hip) at page sizes the parity tests do not
reach.
  python tests/microbench/gzip_leg.py N [PAGE_BYTES]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("", "synth", "kafka-parquet-writer_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import kpw  # noqa: E402
import synth  # noqa: E402

import oracle  # noqa: E402  (the checker)
import pqwalk  # noqa: E402

n = int(sys.argv[1])
page = int(sys.argv[2]) if len(sys.argv) > 2 else 128 << 20
s = synth.REC8
schema = kpw.Schema(s.message_name, s.columns, s.proto_class)
data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE03, n)
props = kpw.ParquetProperties(block_size=128 << 20, compression_codec_name=kpw.GZIP, page_size=page)
for rep in range(2):
    pf = kpw.ParquetFile(None, schema, props)
    t0 = time.perf_counter()
    pf.write_batch((data, offs))
    pf.close()
    dt = time.perf_counter() - t0
    print("gzip writer: %d records (%d bytes), page %d: %.3f s, %.1f MB/s, file %d bytes"
          % (n, int(offs[-1]), page, dt, offs[-1] / dt / 1e6, len(pf.file_bytes())), flush=True)
fb = pf.file_bytes()
t0 = time.perf_counter()
ob = oracle.encode_file(s, data, offs, oracle.make_props(block_size=128 << 20, page_size=page, codec=2))
print("oracle (one core): %.3f s; files identical: %s" % (time.perf_counter() - t0, fb == ob), flush=True)
if fb != ob:
    print(pqwalk.first_difference(fb, ob), flush=True)
    sys.exit(1)
