"""Test infrastructure: the per-record loop alone (C2 Rec8, one kpw_writer_write + one
kpw_writer_data_size per record from C, synth/loop.c), for tracing/profiling.
  python tests/microbench/pr_leg.py N PAGE_BYTES [BLOCK_BYTES]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("", "synth", "kafka-parquet-writer_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))
import kpw  # noqa: E402
import synth  # noqa: E402

if os.environ.get("PR_SPIN") == "1":   # spin-wait synchronisation (hipDeviceScheduleSpin) before any HIP use
    import ctypes
    assert ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(1) == 0
n, page = int(sys.argv[1]), int(sys.argv[2])
block = int(sys.argv[3]) if len(sys.argv) > 3 else 128 << 20
s = synth.REC8
schema = kpw.Schema(s.message_name, s.columns, s.proto_class)
data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE03, n)
props = kpw.ParquetProperties(block_size=block, compression_codec_name=kpw.SNAPPY, page_size=page)
if os.environ.get("PR_WARMUP", "1") != "0":   # first launches load code objects: keep them out
    wf = kpw.ParquetFile(None, schema, props)
    synth.per_record_loop("kpw", wf._L.kpw_writer_write, wf._L.kpw_writer_data_size, wf._h, data, offs, 0,
                          min(n, 50000), 1 << 62)
    wf.close()
pf = kpw.ParquetFile(None, schema, props)
L = pf._L
t0 = time.perf_counter()
got, full, st, last = synth.per_record_loop("kpw", L.kpw_writer_write, L.kpw_writer_data_size, pf._h, data, offs, 0, n, 1 << 62)
dt = time.perf_counter() - t0
assert (got, st) == (n, 0), (got, st)
pf.close()
print("per-record loop: %d records, page %d, block %d: %.3f s, %.2f M records/s, file %d bytes"
      % (n, page, block, dt, n / dt / 1e6, len(pf.file_bytes())), flush=True)
