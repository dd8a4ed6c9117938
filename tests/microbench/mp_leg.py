"""Test infrastructure: the bulk multi-page writer leg alone (C2 Rec8, 128 MiB row groups,
PAGE-byte pages, pinned poll batches through kpw_writer_write_async), for tracing/profiling.
  python tests/microbench/mp_leg.py N PAGE_BYTES [STEPS]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("", "synth", "kafka-parquet-writer_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))
import kpw  # noqa: E402
import synth  # noqa: E402

n, page = int(sys.argv[1]), int(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
s = synth.REC8
schema = kpw.Schema(s.message_name, s.columns, s.proto_class)
data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE02, n, alloc=kpw.pinned_empty)
props = kpw.ParquetProperties(block_size=128 << 20, compression_codec_name=kpw.SNAPPY, page_size=page)
for i in range(steps):
    t0 = time.perf_counter()
    pf = kpw.ParquetFile(None, schema, props)
    for a in range(0, n, 500_000):
        b = min(n, a + 500_000)
        pf._check(pf._L.kpw_writer_write_async(pf._h, data.ctypes.data, offs.ctypes.data + 8 * a, b - a), "write")
    pf.close()
    dt = time.perf_counter() - t0
    print("step %d: %d records, page %d: %.1f ms, %.2f GB/s, file %d bytes" % (i, n, page, dt * 1e3, int(offs[-1]) / dt / 1e9,
                                                                            len(pf.file_bytes())), flush=True)
    del pf
