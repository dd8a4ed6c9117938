"""Test infrastructure (run by test_gpu_multipage.py in a child process, so that KPW_EAGER_MB,
read once per process, can be small): bulk multi-page writes through the ParquetFile drop-in,
each batch large enough to submit an eager write-path job, which leaves its open row group to
the next job (Engine::lazy_open).  argv: mode ("file" | "data_size"), codec."""
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
mode, codec = sys.argv[1], int(sys.argv[2])
n, batch = 1_500_000, 100_000
data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE45, n)
props = kpw.ParquetProperties(block_size=4 * MiB, page_size=64 * 1024, compression_codec_name=codec)
oprops = oracle.make_props(block_size=4 * MiB, page_size=64 * 1024, codec=codec)
pf = kpw.ParquetFile(None, kpw.Schema(synth.REC8.message_name, synth.REC8.columns, synth.REC8.proto_class), props)
ow = oracle.OracleWriter(synth.REC8, oprops) if mode == "data_size" else None
for a in range(0, n, batch):
    b = min(n, a + batch)
    pf.write_batch((data[int(offs[a]):int(offs[b])], (offs[a:b + 1] - offs[a]).astype(np.uint64)))
    if ow is not None:
        st, nw = ow.write_batch(data, offs[a:b + 1])
        assert st == 0 and nw == b - a, (st, nw)
        # the first getDataSize comes after three batches, so it finds a lazy job's unknown open
        # row group; from then on the writer plans every job's open row group (size_polled)
        if a >= 3 * batch:
            got, want = pf.get_data_size(), ow.data_size()
            assert got == want, (a, got, want)
pf.close()
fb = pf.file_bytes()
ob = oracle.encode_file(synth.REC8, data, offs, oprops)
assert fb == ob, pqwalk.first_difference(fb, ob)
print("LAZY_OPEN_OK", len(pqwalk.footer(fb)[4]), "row groups")
