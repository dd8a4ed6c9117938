"""File rotation on the GPU path: kpw_writer_write_until_full against the oracle's WorkerThread
loop (KafkaProtoParquetWriter.java:268-285,306-308: write one record, rotate right after the
first record for which getDataSize() >= maxFileSize).  Bar: the same number of records in
every file and byte-identical files; the reference's own expectation
(KafkaProtoParquetWriterTest.java:142-174, 0.9 < maxFileSize / len < 1.01) also holds."""
import io

import numpy as np
import pyarrow.parquet as pq
import pytest

import oracle
import synth

pytestmark = pytest.mark.gpu
MiB = 1024 * 1024


def _rotate(schema, data, offs, max_file, block_size, codec, chunk, writer_version=1, max_files=4):
    """Write files until the records run out; each call hands `chunk` records (the rest of the
    file's records stay with the caller, as a poll() batch would)."""
    import kpw
    props = kpw.ParquetProperties(block_size=block_size, compression_codec_name=codec, writer_version=writer_version)
    oprops = oracle.make_props(block_size=block_size, codec=codec, writer_version=writer_version)
    n = len(offs) - 1
    start = 0
    files = []
    while start < n and len(files) < max_files:
        pf = kpw.ParquetFile(None, kpw.Schema(schema.message_name, schema.columns, schema.proto_class), props)
        ow = oracle.OracleWriter(schema, oprops)
        pos, full = start, False
        while pos < n and not full:
            end = min(n, pos + chunk)
            sub = (offs[pos:end + 1] - offs[pos]).astype(np.uint64)
            seg = data[int(offs[pos]):int(offs[end])]
            na, full = pf.write_until_full((seg, sub), max_file)
            st, ona, ofull = ow.write_until_full(seg, sub, max_file)
            assert st == 0
            assert (na, full) == (ona, bool(ofull)), (start, pos, na, full, ona, ofull)
            assert pf.get_data_size() == ow.data_size()
            pos += na
        pf.close()
        ow.close()
        fb, ob = pf.file_bytes(), ow.file_bytes()
        import pqwalk
        assert fb == ob, pqwalk.first_difference(fb, ob)
        files.append((fb, full))
        start = pos
    return files


@pytest.mark.parametrize("codec", [0, 1], ids=["uncompressed", "snappy"])
def test_max_file_size_reference_case(codec):
    """testMaxFileSize restated: 10 KiB row groups, maxFileSize 100 KiB."""
    data, offs = synth.generate(synth.KIND_SAMPLE, 0xC0FFEE01, 12000)
    files = _rotate(synth.SAMPLE, data, offs, 100 * 1024, 10 * 1024, codec, chunk=12000)
    full = [fb for fb, f in files if f]
    assert len(full) >= 2
    for fb in full:
        assert 0.9 < 100 * 1024 / len(fb) < 1.01
        assert pq.read_table(io.BytesIO(fb)).num_rows > 0


@pytest.mark.parametrize("chunk", [700, 5000], ids=["chunk700", "chunk5000"])
def test_rotation_rec8_chunked(chunk):
    """Several calls per file: records staged by earlier calls stay in the open row group."""
    data, offs = synth.generate(synth.KIND_REC8, 41, 40000)
    files = _rotate(synth.REC8, data, offs, 600 * 1024, 64 * 1024, 1, chunk=chunk)
    assert sum(1 for _, f in files if f) >= 2


def test_rotation_v2():
    data, offs = synth.generate(synth.KIND_SAMPLE, 43, 12000, param=30)
    files = _rotate(synth.SAMPLE, data, offs, 80 * 1024, 8 * 1024, 1, chunk=3000, writer_version=2)
    assert sum(1 for _, f in files if f) >= 2


def test_rotation_highcard_fallback():
    data, offs = synth.generate(synth.KIND_HIGHCARD, 44, 6000)
    files = _rotate(synth.HIGHCARD, data, offs, 400 * 1024, 128 * 1024, 1, chunk=2500)
    assert files


def test_data_size_per_record():
    """getDataSize() after every record (the reference's own check, KPW:306-308)."""
    import kpw
    data, offs = synth.generate(synth.KIND_SAMPLE, 45, 260)
    props = kpw.ParquetProperties(block_size=2 * 1024, compression_codec_name=1)
    pf = kpw.ParquetFile(None, kpw.Schema(synth.SAMPLE.message_name, synth.SAMPLE.columns, synth.SAMPLE.proto_class),
                         props)
    ow = oracle.OracleWriter(synth.SAMPLE, oracle.make_props(block_size=2 * 1024, codec=1))
    for i in range(260):
        sub = np.array([0, offs[i + 1] - offs[i]], dtype=np.uint64)
        seg = data[int(offs[i]):int(offs[i + 1])]
        pf.write_batch((seg, sub))
        ow.write_batch(seg, sub)
        assert pf.get_data_size() == ow.data_size(), i
    pf.close()
    ow.close()
    import pqwalk
    assert pf.file_bytes() == ow.file_bytes(), pqwalk.first_difference(pf.file_bytes(), ow.file_bytes())


def test_multipage_regime_unsupported():
    import kpw
    props = kpw.ParquetProperties(block_size=1 * MiB, page_size=64 * 1024)
    pf = kpw.ParquetFile(None, kpw.Schema(synth.SAMPLE.message_name, synth.SAMPLE.columns), props)
    data, offs = synth.generate(synth.KIND_SAMPLE, 46, 10)
    with pytest.raises(kpw.KpwError):
        pf.write_until_full((data, offs), 1000)
    pf.close()


def _writer_lib():
    import kpw
    return kpw.load_library()


def test_data_size_every_record_200k():
    """The reference's unchanged WorkerThread loop (KafkaProtoParquetWriter.java:268-285,306-308):
    ParquetFile.write of ONE record, then getDataSize(), 200 000 times.  Every value equals the
    oracle's InternalParquetRecordWriter.getDataSize(), row groups are cut on the host by the size
    model (one GPU encode per row group), and the file is byte-identical."""
    import ctypes
    import time
    import kpw
    import pqwalk
    n = 200_000
    data, offs = synth.generate(synth.KIND_REC8, 47, n)
    props = kpw.ParquetProperties(block_size=1 * MiB, compression_codec_name=1)
    pf = kpw.ParquetFile(None, kpw.Schema(synth.REC8.message_name, synth.REC8.columns, synth.REC8.proto_class), props)
    ow = oracle.OracleWriter(synth.REC8, oracle.make_props(block_size=1 * MiB, codec=1))
    L, OL = pf._L, oracle.lib()
    base = data.ctypes.data
    one = np.zeros(2, dtype=np.uint64)
    optr = one.ctypes.data
    got = np.empty(n, dtype=np.int64)
    want = np.empty(n, dtype=np.int64)
    t0 = time.perf_counter()
    for i in range(n):
        a, b = int(offs[i]), int(offs[i + 1])
        one[1] = b - a
        assert L.kpw_writer_write(pf._h, base + a, optr, 1) == 0
        got[i] = L.kpw_writer_data_size(pf._h)
    dt = time.perf_counter() - t0
    for i in range(n):
        a, b = int(offs[i]), int(offs[i + 1])
        assert OL.kpwo_write(ow._h, base + a, b - a) == 0
        want[i] = ow.data_size()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (int(bad[0]), int(got[bad[0]]), int(want[bad[0]]))
    assert ow.num_row_groups() >= 8
    pf.close()
    ow.close()
    assert pf.file_bytes() == ow.file_bytes(), pqwalk.first_difference(pf.file_bytes(), ow.file_bytes())
    assert dt < 30, dt


def test_rotation_per_record_model():
    """write_until_full one record at a time (model path) across files."""
    data, offs = synth.generate(synth.KIND_REC8, 48, 30000)
    files = _rotate(synth.REC8, data, offs, 300 * 1024, 32 * 1024, 1, chunk=1)
    assert sum(1 for _, f in files if f) >= 2


def test_bulk_then_per_record():
    """A bulk write (> 65536 records: GPU-planned cuts) and then one-record writes with
    getDataSize() after each (the GPU answers from the staged records)."""
    import kpw
    import pqwalk
    data, offs = synth.generate(synth.KIND_SAMPLE, 49, 70200)
    props = kpw.ParquetProperties(block_size=256 * 1024, compression_codec_name=1)
    pf = kpw.ParquetFile(None, kpw.Schema(synth.SAMPLE.message_name, synth.SAMPLE.columns, synth.SAMPLE.proto_class),
                         props)
    ow = oracle.OracleWriter(synth.SAMPLE, oracle.make_props(block_size=256 * 1024, codec=1))
    pf.write_batch((data[:int(offs[70000])], offs[:70001]))
    ow.write_batch(data, offs[:70001])
    assert pf.get_data_size() == ow.data_size()
    for i in range(70000, 70200):
        sub = np.array([0, offs[i + 1] - offs[i]], dtype=np.uint64)
        seg = data[int(offs[i]):int(offs[i + 1])]
        pf.write_batch((seg, sub))
        ow.write_batch(seg, sub)
        assert pf.get_data_size() == ow.data_size(), i
    pf.close()
    ow.close()
    assert pf.file_bytes() == ow.file_bytes(), pqwalk.first_difference(pf.file_bytes(), ow.file_bytes())


def test_pinned_source_bulk():
    """Batches in kpw_host_alloc memory are DMA'd directly (no host copy); same file bytes."""
    import kpw
    import pqwalk
    data, offs = synth.generate(synth.KIND_REC8, 50, 400000)
    pin = kpw.pinned_empty(len(data))
    pin[:] = data
    props = kpw.ParquetProperties(block_size=2 * MiB, compression_codec_name=1)
    pf = kpw.ParquetFile(None, kpw.Schema(synth.REC8.message_name, synth.REC8.columns, synth.REC8.proto_class), props)
    for a, b in ((0, 150000), (150000, 300000), (300000, 400000)):
        pf.write_batch((pin[int(offs[a]):int(offs[b])], (offs[a:b + 1] - offs[a]).astype(np.uint64)))
    pf.close()
    want = oracle.encode_file(synth.REC8, data, offs, oracle.make_props(block_size=2 * MiB, codec=1))
    assert pf.file_bytes() == want, pqwalk.first_difference(pf.file_bytes(), want)


@pytest.mark.parametrize("codec", [0, 1], ids=["uncompressed", "snappy"])
def test_rotation_bulk_path(codec):
    """write_until_full with poll()-sized batches of > 65536 records (the GPU-planned bulk path:
    one full encode per call, plan-only probes inside the crossing row group) against the
    oracle's record-at-a-time loop: same records per file, byte-identical files."""
    data, offs = synth.generate(synth.KIND_REC8, 45, 330000)
    files = _rotate(synth.REC8, data, offs, 3 * MiB, 256 * 1024, codec, chunk=100000, max_files=6)
    assert sum(1 for _, f in files if f) >= 2
