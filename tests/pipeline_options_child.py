"""Test infrastructure (run by test_gpu_options.py in a child process, so that environment
knobs read once per process can be set): writer pipeline options that the default runs do not
take, each checked against the oracle.  argv: mode.
  probe_exact  KPW_PROBE_EXACT=1: the page-size probes' dictionary continuation compares string
               keys byte for byte from a row group's first probe (the path a 64-bit hash
               collision switches to); every getDataSize of a per-record loop with 64 KiB pages
               and the file must equal the oracle's
  gate         KPW_DEVICE_ENCODES=1: three concurrent writers whose jobs are admitted one at a
               time (small eager / full jobs: many jobs per file)
  encoders3    KPW_ENCODERS=3: three encode workers per writer, small jobs"""
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "synth"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "kafka-parquet-writer_amd"), ROOT]
import numpy as np  # noqa: E402

import kpw  # noqa: E402
import oracle  # noqa: E402
import pqwalk  # noqa: E402
import synth  # noqa: E402

MiB = 1024 * 1024
mode = sys.argv[1]
S = synth.REC8
schema = kpw.Schema(S.message_name, S.columns, S.proto_class)


def bulk_file(seed, n):
    data, offs = synth.generate(synth.KIND_REC8, seed, n)
    props = kpw.ParquetProperties(block_size=4 * MiB, compression_codec_name=1)
    pf = kpw.ParquetFile(None, schema, props)
    for a in range(0, n, 50_000):
        b = min(n, a + 50_000)
        pf.write_batch((data[int(offs[a]):int(offs[b])], (offs[a:b + 1] - offs[a]).astype(np.uint64)))
    pf.close()
    fb = pf.file_bytes()
    ob = oracle.encode_file(S, data, offs, oracle.make_props(block_size=4 * MiB, codec=1))
    assert fb == ob, (seed, pqwalk.first_difference(fb, ob))
    return pf.pipeline_stats()


if mode == "probe_exact":
    assert os.environ.get("KPW_PROBE_EXACT") == "1"
    n = 60_000
    data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE71, n)
    props = kpw.ParquetProperties(block_size=4 * MiB, page_size=64 * 1024, compression_codec_name=1)
    pf = kpw.ParquetFile(None, schema, props)
    ow = oracle.OracleWriter(S, oracle.make_props(block_size=4 * MiB, page_size=64 * 1024, codec=1))
    L, OL = pf._L, oracle.lib()
    base = data.ctypes.data
    one = np.zeros(2, dtype=np.uint64)
    got = np.empty(n, dtype=np.int64)
    want = np.empty(n, dtype=np.int64)
    for i in range(n):
        a, b = int(offs[i]), int(offs[i + 1])
        one[1] = b - a
        assert L.kpw_writer_write(pf._h, base + a, one.ctypes.data, 1) == 0
        got[i] = L.kpw_writer_data_size(pf._h)
        assert OL.kpwo_write(ow._h, base + a, b - a) == 0
        want[i] = ow.data_size()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (int(bad[0]), int(got[bad[0]]), int(want[bad[0]]))
    pf.close()
    ow.close()
    assert pf.file_bytes() == ow.file_bytes(), pqwalk.first_difference(pf.file_bytes(), ow.file_bytes())
    print("OPTIONS_OK probe_exact", n, "records")
elif mode == "gate":
    assert os.environ.get("KPW_DEVICE_ENCODES") == "1"
    res, errs = [None] * 3, []

    def one_writer(k):
        try:
            res[k] = bulk_file(0xC0FFEE72 + k, 300_000)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=one_writer, args=(k,)) for k in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs[0]
    jobs = sum(r["jobs"] for r in res)
    assert jobs >= 6, jobs
    print("OPTIONS_OK gate", int(jobs), "jobs")
elif mode == "encoders3":
    assert os.environ.get("KPW_ENCODERS") == "3"
    st = bulk_file(0xC0FFEE75, 400_000)
    assert st["jobs"] >= 3, st["jobs"]
    print("OPTIONS_OK encoders3", int(st["jobs"]), "jobs")
else:
    raise SystemExit("unknown mode " + mode)
