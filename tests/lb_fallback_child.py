"""Test infrastructure (run by test_gpu_lookback.py in a child process, so that KPW_LB_SPIN,
read once per process, can be 0): every single-pass look-back scan (kpw_lookback.h) that does
not find its predecessor's status at the first poll recomputes it (the decoupled fallback),
so the fallbacks of k_seg_scan, k_phase (both scans) and k_r_sizes run on real encodes.  Each
file must still be byte-identical to the oracle's, and fallbacks must have been taken."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "synth"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "kafka-parquet-writer_amd"), ROOT]
import numpy as np  # noqa: E402

import kpw  # noqa: E402
import oracle  # noqa: E402
import pqwalk  # noqa: E402
import synth  # noqa: E402

MiB = 1024 * 1024
assert os.environ.get("KPW_LB_SPIN") == "0"
cases = [
    # kind, n, seed, page_size, writer_version
    (synth.KIND_REC8, 400_000, 0xC0FFEE61, 128 * MiB, 1),
    (synth.KIND_REC8, 400_000, 0xC0FFEE62, 64 * 1024, 1),     # multi-page regime
    (synth.KIND_HIGHCARD, 300_000, 0xC0FFEE63, 128 * MiB, 1),
    (synth.KIND_WIDE, 40_000, 0xC0FFEE64, 128 * MiB, 1),
    (synth.KIND_HIGHCARD, 200_000, 0xC0FFEE65, 128 * MiB, 2),   # v2: DELTA encodings' scans
]
total_fb = 0
for kind, n, seed, page_size, wv in cases:
    schema = synth.SCHEMAS[kind]
    data, offs = synth.generate(kind, seed, n)
    props = kpw.ParquetProperties(page_size=page_size, compression_codec_name=1, writer_version=wv)
    pf = kpw.ParquetFile(None, kpw.Schema(schema.message_name, schema.columns, schema.proto_class), props)
    batch = 100_000
    for a in range(0, n, batch):
        b = min(n, a + batch)
        pf.write_batch((data[int(offs[a]):int(offs[b])], (offs[a:b + 1] - offs[a]).astype(np.uint64)))
    pf.close()
    fbk = pf.pipeline_stats().get("lookback_fallbacks", 0)
    fb = pf.file_bytes()
    ob = oracle.encode_file(schema, data, offs, oracle.make_props(page_size=page_size, codec=1, writer_version=wv))
    assert fb == ob, (schema.message_name, page_size, wv, pqwalk.first_difference(fb, ob))
    print(schema.message_name, page_size, wv, "fallbacks", int(fbk))
    total_fb += int(fbk)
assert total_fb > 0, "no look-back fell back"
print("LB_FALLBACK_OK", total_fb)
