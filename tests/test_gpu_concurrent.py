"""C5 shape on one GPU: concurrent writers (BASELINE config 5).

The reference runs `threadCount` WorkerThreads, each owning one open ParquetFile
(KafkaProtoParquetWriter.java:175-179,216-240); ParquetFile is not thread-safe but separate
instances are used from separate threads (ParquetFile.java:19-20).  Here several kpw_writer
handles on the same device are driven from their own threads at once (ctypes releases the
GIL inside the C-ABI), each on its own Kafka partition (seed 0xC0FFEE05 + p), half through
the per-record size-model path and half through the bulk path; every file must be
byte-identical to the oracle's file of the same records.
"""
import threading

import numpy as np
import pytest

import oracle
import pqwalk
import synth

pytestmark = pytest.mark.gpu
MiB = 1024 * 1024


def _write_partition(p, n, batch, out, errs):
    import kpw
    try:
        data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE05 + p, n)
        props = kpw.ParquetProperties(block_size=1 * MiB, compression_codec_name=1)
        pf = kpw.ParquetFile(None, kpw.Schema(synth.REC8.message_name, synth.REC8.columns, synth.REC8.proto_class),
                             props)
        sizes = []
        for a in range(0, n, batch):
            b = min(n, a + batch)
            pf.write_batch((data[int(offs[a]):int(offs[b])], (offs[a:b + 1] - offs[a]).astype(np.uint64)))
            sizes.append(pf.get_data_size())
        pf.close()
        out[p] = (pf.file_bytes(), data, offs, sizes)
    except Exception as e:  # noqa: BLE001
        errs.append((p, e))


@pytest.mark.parametrize("writers", [4, 8])
def test_concurrent_writers_one_device(writers):
    n = 150_000
    out, errs = {}, []
    ts = [threading.Thread(target=_write_partition, args=(p, n, 5_000 if p % 2 == 0 else 75_000, out, errs))
          for p in range(writers)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    for p in range(writers):
        fb, data, offs, sizes = out[p]
        ow = oracle.OracleWriter(synth.REC8, oracle.make_props(block_size=1 * MiB, codec=1))
        batch = 5_000 if p % 2 == 0 else 75_000
        want_sizes = []
        for a in range(0, n, batch):
            b = min(n, a + batch)
            st, _ = ow.write_batch(data, offs[a:b + 1])
            assert st == 0
            want_sizes.append(ow.data_size())
        ow.close()
        assert sizes == want_sizes, p
        assert fb == ow.file_bytes(), (p, pqwalk.first_difference(fb, ow.file_bytes()))
