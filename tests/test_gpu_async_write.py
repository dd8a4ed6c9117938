"""kpw_writer_write_async: a consumer polling into a ring of two pinned batches (north_star:
polled batches in pinned staging, moved to HBM on a side stream).  A ring slot is refilled
right after the call that followed its write returned, which the contract allows; the file
must still be byte-identical to the oracle's (ParquetFile.java:59-68 restated), whatever the
DMA timing."""
import numpy as np
import pytest

import oracle
import pqwalk
import synth

pytestmark = pytest.mark.gpu
MiB = 1024 * 1024


@pytest.mark.parametrize("batch", [100_000, 250_000])
def test_async_ring_of_two_pinned_batches(batch):
    import kpw
    n = 1_200_000
    data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE0A, n)
    cap = max(int(offs[min(n, a + batch)] - offs[a]) for a in range(0, n, batch))
    ring = [kpw.pinned_empty(cap), kpw.pinned_empty(cap)]
    props = kpw.ParquetProperties(block_size=4 * MiB, compression_codec_name=kpw.SNAPPY)
    pf = kpw.ParquetFile(None, kpw.Schema(synth.REC8.message_name, synth.REC8.columns, synth.REC8.proto_class), props)
    for k, a in enumerate(range(0, n, batch)):
        b = min(n, a + batch)
        slot = ring[k % 2]
        ln = int(offs[b] - offs[a])
        slot[:ln] = data[int(offs[a]):int(offs[b])]   # the slot's previous batch was released
        slot[ln:ln + 64] = 0xEE                         # (garbage after the batch)
        pf.write_batch_async(slot, offs[a:b + 1] - offs[a])
    pf.close()
    fb = pf.file_bytes()
    want = oracle.encode_file(synth.REC8, data, offs, oracle.make_props(block_size=4 * MiB, codec=1))
    assert fb == want, pqwalk.first_difference(fb, want)
    assert pf.get_num_written_records() == n


def test_async_then_sync_calls_release_the_batch():
    """getDataSize and a plain write after an async write wait for its DMA (the batch may be
    reused once they return)."""
    import kpw
    n = 400_000
    data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE0B, n)
    half = n // 2
    buf = kpw.pinned_empty(int(offs[half]))
    buf[:] = data[:int(offs[half])]
    props = kpw.ParquetProperties(block_size=2 * MiB, compression_codec_name=kpw.SNAPPY)
    pf = kpw.ParquetFile(None, kpw.Schema(synth.REC8.message_name, synth.REC8.columns, synth.REC8.proto_class), props)
    pf.write_batch_async(buf, offs[:half + 1])
    ds = pf.get_data_size()
    buf[:] = 0x5A   # released by getDataSize()
    pf.write_batch((data[int(offs[half]):], offs[half:] - offs[half]))
    pf.close()
    ow = oracle.OracleWriter(synth.REC8, oracle.make_props(block_size=2 * MiB, codec=1))
    st, _ = ow.write_batch(data, offs[:half + 1])
    assert st == 0 and ow.data_size() == ds
    st, _ = ow.write_batch(data, offs[half:])
    assert st == 0
    ow.close()
    assert pf.file_bytes() == ow.file_bytes()


@pytest.mark.parametrize("getter", ["num_records", "creation_time", "failed_record", "last_error"])
def test_async_then_getter_releases_the_batch(getter):
    """Every kpw_writer_* entry point releases an async write's batch: a consumer
    that calls getNumWrittenRecords() (or another getter) after kpw_writer_write_async and then
    refills the slot must not corrupt the file."""
    import kpw
    n = 600_000
    data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE0C, n)
    third = n // 3
    buf = kpw.pinned_empty(int(offs[third]))
    buf[:] = data[:int(offs[third])]
    props = kpw.ParquetProperties(block_size=2 * MiB, compression_codec_name=kpw.SNAPPY)
    pf = kpw.ParquetFile(None, kpw.Schema(synth.REC8.message_name, synth.REC8.columns, synth.REC8.proto_class), props)
    pf.write_batch_async(buf, offs[:third + 1])
    L, h = pf._L, pf._h
    {"num_records": L.kpw_writer_num_records, "creation_time": L.kpw_writer_creation_time_ms,
     "failed_record": L.kpw_writer_failed_record, "last_error": L.kpw_writer_last_error}[getter](h)
    buf[:] = 0x5A   # released by the getter
    pf.write_batch((data[int(offs[third]):], offs[third:] - offs[third]))
    pf.close()
    want = oracle.encode_file(synth.REC8, data, offs, oracle.make_props(block_size=2 * MiB, codec=1))
    assert pf.file_bytes() == want, pqwalk.first_difference(pf.file_bytes(), want)
