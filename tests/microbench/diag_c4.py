"""Test infrastructure: isolate the C4 row-group-1 blob mismatch.  Modes:
  enc N      - kpw.Encoder on the first N records resident in HBM, pages vs the oracle
  writer N   - the ParquetFile writer path on the first N records (500 k poll batches)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("", "tests", "synth", "kafka-parquet-writer_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402

import gpu_helpers  # noqa: E402
import kpw  # noqa: E402
import oracle  # noqa: E402
import synth  # noqa: E402

MiB = 1024 * 1024
mode, n = sys.argv[1], int(sys.argv[2])
schema = synth.SCHEMAS[synth.KIND_HIGHCARD]
data, offs = synth.generate(synth.KIND_HIGHCARD, 0xC0FFEE04, n)
props = oracle.make_props(block_size=128 * MiB, page_size=128 * MiB, codec=0, enable_dictionary=True)
if mode == "enc":
    errs = gpu_helpers.compare_pages(schema, data, offs, codec=0)
    print("encoder path, %d records: %d mismatches %s" % (n, len(errs), errs[:4]))
else:
    pf = kpw.ParquetFile(None, kpw.Schema(schema.message_name, schema.columns, schema.proto_class),
                         kpw.ParquetProperties(compression_codec_name=0))
    for a in range(0, n, 500_000):
        b = min(n, a + 500_000)
        pf.write_batch((data[int(offs[a]):int(offs[b])], (offs[a:b + 1] - offs[a]).astype(np.uint64)))
    pf.close()
    fb = pf.file_bytes()
    errs = gpu_helpers.check_row_groups(schema, data, offs, fb, props)
    print("writer path, %d records, env %s: %d mismatches %s" % (
        n, {k: v for k, v in os.environ.items() if k.startswith("KPW_")}, len(errs), errs[:4]))
sys.stdout.flush()
