"""GPU properties at the bench's full size (C2: 100 M Rec8 records, 49 row groups; SURVEY.md
§8d), where the CPU oracle would need minutes.  Size-independent checks instead of a byte
comparison with the oracle (which test_gpu_parity.py does at smaller sizes):
  - Snappy round trip: every page of a SNAPPY encode decompresses (pyarrow's Snappy) to the
    same page of an UNCOMPRESSED encode of the same batch, and the uncompressed sizes agree;
  - structure: the row groups tile [0, n) in order and every chunk holds its row group's
    records;
  - file readback: the file written through the ParquetFile mirror reads back in pyarrow with
    n rows, and every column chunk's footer statistics (null count, min, max) equal what
    pyarrow computes from the values it decoded.
KPW_FULL_N overrides the record count (default: the bench's 100 M)."""
import os

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu
N = int(os.environ.get("KPW_FULL_N", 100_000_000))
SEED = 0xC0FFEE02   # bench.py's C2 seed


@pytest.fixture(scope="module")
def c2():
    import kpw
    data, offs = synth.generate(synth.KIND_REC8, SEED, N)
    d = kpw.DeviceBuffer.from_array(data)   # HBM from the library's own HIP runtime
    o = kpw.DeviceBuffer.from_array(offs.astype(np.uint64))
    yield data, offs, d, o
    d.free()
    o.free()


def _encode(d, o, codec):
    import kpw
    s = synth.REC8
    enc = kpw.Encoder(kpw.Schema(s.message_name, s.columns, s.proto_class), codec=codec)
    enc.encode(d.ptr, o.ptr, N, final=True)
    return enc


def test_full_size_snappy_roundtrip(c2):
    import pyarrow as pa
    _, _, d, o = c2
    e0 = _encode(d, o, 0)
    rg0, p0, ch0, b0 = e0.row_groups(), e0.pages(), e0.chunks(), e0.pages_bytes()
    del e0
    e1 = _encode(d, o, 1)
    rg1, p1, b1 = e1.row_groups(), e1.pages(), e1.pages_bytes()
    del e1
    # structure
    assert rg0 == rg1 and len(rg0) > 1
    start = 0
    for first, cnt in rg0:
        assert first == start and cnt > 0
        start += cnt
    assert start == N
    ncols = len(synth.REC8.columns)
    assert len(ch0) == len(rg0) * ncols
    for k, c in enumerate(ch0):
        assert c["num_values"] == rg0[k // ncols][1]
    # Snappy round trip, page by page
    assert len(p0) == len(p1)
    raw_total = 0
    for x, y in zip(p0, p1):
        assert (x["page_type"], x["num_values"], x["uncompressed_size"]) == (y["page_type"], y["num_values"],
                                                                             y["uncompressed_size"])
        raw = b0[x["offset"]:x["offset"] + x["compressed_size"]]
        comp = b1[y["offset"]:y["offset"] + y["compressed_size"]]
        assert len(raw) == x["uncompressed_size"]
        got = pa.decompress(comp, decompressed_size=len(raw), codec="snappy", asbytes=True) if raw else b""
        assert got == raw
        raw_total += len(raw)
    assert raw_total > N   # sanity: pages hold at least a byte per record


def test_full_size_file_readback(c2):
    import io

    import pyarrow.compute as pc
    import pyarrow.parquet as pq

    import kpw
    data, offs, _, _ = c2
    s = synth.REC8
    pf = kpw.ParquetFile(None, kpw.Schema(s.message_name, s.columns, s.proto_class),
                         kpw.ParquetProperties(compression_codec_name=kpw.SNAPPY))
    pf.write_batch((data, offs))
    pf.close()
    fb = pf.file_bytes()
    del pf
    f = pq.ParquetFile(io.BytesIO(fb))
    md = f.metadata
    assert md.num_rows == N
    names = [c[0] for c in s.columns]
    for rg in range(md.num_row_groups):
        t = f.read_row_group(rg)
        assert t.num_rows == md.row_group(rg).num_rows
        for ci, name in enumerate(names):
            col = t.column(name)
            st = md.row_group(rg).column(ci).statistics
            assert st is not None and st.has_null_count
            assert st.null_count == col.null_count, (rg, name)
            if col.null_count == len(col) or not st.has_min_max:
                continue
            mm = pc.min_max(col)
            assert st.min == mm["min"].as_py(), (rg, name)
            assert st.max == mm["max"].as_py(), (rg, name)
