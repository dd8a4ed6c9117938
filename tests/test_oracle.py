"""Pins the CPU oracle before anything is compared against it.

- hand-derived known-answer vectors (tests/golden/spec_vectors.json);
- pyarrow 25 reads every oracle file back value-exact (vs google.protobuf's own parse);
- pyarrow's Snappy decodes every page the oracle compresses;
- the reference test's record-level assertions restated (KafkaProtoParquetWriterTest.java).
"""
import io
import json
import os
import struct

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

import oracle
import pqwalk
import protoutil
import synth
import wire_cases

HERE = os.path.dirname(os.path.abspath(__file__))
SPEC = json.load(open(os.path.join(HERE, "golden", "spec_vectors.json")))
MiB = 1024 * 1024


@pytest.mark.parametrize("vec", SPEC["rle_hybrid"], ids=lambda v: v["name"])
def test_rle_known_answers(vec):
    assert oracle.rle_encode(vec["values"], vec["bit_width"]).hex().upper() == vec["expected_hex"]


@pytest.mark.parametrize("vec", SPEC["snappy"], ids=lambda v: v["name"])
def test_snappy_known_answers(vec):
    assert oracle.snappy_compress(bytes.fromhex(vec["input_hex"])).hex() == vec["expected_hex"].lower()


@pytest.mark.parametrize("n", [1, 14, 15, 16, 100, 4096, 65535, 65536, 65537, 200000])
def test_snappy_roundtrip_pyarrow(n):
    rng = np.random.default_rng(n)
    for kind in range(3):
        if kind == 0:
            data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif kind == 1:
            data = (b"kafka-parquet-" * (n // 14 + 1))[:n]
        else:
            data = rng.integers(0, 4, n, dtype=np.uint8).tobytes()
        c = oracle.snappy_compress(data)
        assert pa.decompress(c, decompressed_size=n, codec="snappy", asbytes=True) == data


def _zlib_gzip_member(data):
    """What GzipCodec without native hadoop writes per page: java.util.zip.GZIPOutputStream
    (Java 8) = header 1f 8b 08 00, MTIME 0, XFL 0, OS 0 + zlib level-6 raw deflate (here: Python's
    zlib, the same zlib 1.2.11 algorithm) + CRC-32 + ISIZE."""
    import zlib
    c = zlib.compressobj(6, zlib.DEFLATED, -15, 8, zlib.Z_DEFAULT_STRATEGY)
    body = c.compress(data) + c.flush()
    return bytes([0x1F, 0x8B, 8, 0, 0, 0, 0, 0, 0, 0]) + body + struct.pack("<II", zlib.crc32(data), len(data) & 0xFFFFFFFF)


def _deflate_inputs():
    rng = np.random.default_rng(11)
    out = [b"", b"a", b"ab", b"abc", b"aaaa", bytes(1), bytes(300), bytes(70000)]
    out.append(rng.integers(0, 256, 150_000, dtype=np.uint8).tobytes())          # stored blocks
    out.append(rng.integers(0, 3, 250_000, dtype=np.uint8).tobytes())            # long chains, window slides
    out.append((b"kafka-parquet-writer gzip page " * 9000)[:200_000])           # long matches
    out.append(b"".join(struct.pack("<q", 1_700_000_000_000 + i + int(v)) for i, v in
                        enumerate(rng.integers(0, 1000, 40_000))))                # PLAIN int64
    js = b"".join(b'{"id":%d,"event":"%s","value":%d}' % (i, b"click" if v & 1 else b"view", v % 99991)
                  for i, v in enumerate(rng.integers(0, 1 << 30, 12_000)))
    out.append(js)                                                               # lazy matches, dynamic trees
    out.append(bytes(rng.integers(0, 256, 40_000, dtype=np.uint8)) + bytes(40_000) + js[:50_000])   # mixed blocks
    return out


@pytest.mark.parametrize("i", range(14))
def test_deflate_matches_zlib(i):
    """The oracle's deflate (a restatement of zlib 1.2.11 level 6) is byte-identical to the zlib
    Python links, and each page member round-trips through the gzip module."""
    import gzip
    data = _deflate_inputs()[i]
    assert oracle.gzip_compress(data) == _zlib_gzip_member(data)
    assert gzip.decompress(oracle.gzip_compress(data)) == data


def test_deflate_matches_zlib_16mib():
    """A 16 MiB input (hundreds of window slides, ~1000 blocks): text, PLAIN int64, zero runs,
    incompressible stretches and JSON, interleaved in 1 MiB pieces, byte-identical to zlib."""
    import gzip
    rng = np.random.default_rng(16)
    parts = []
    ins = _deflate_inputs()
    for k in range(16):
        m = k % 4
        if m == 0:
            parts.append((ins[12] * 6)[:MiB])
        elif m == 1:
            parts.append(np.cumsum(rng.integers(0, 5000, MiB // 8), dtype=np.int64).astype("<i8").tobytes())
        elif m == 2:
            parts.append(bytes(MiB // 2) + rng.integers(0, 256, MiB // 2, dtype=np.uint8).tobytes())
        else:
            parts.append(rng.integers(0, 7, MiB, dtype=np.uint8).tobytes())
    data = b"".join(parts)
    assert len(data) == 16 * MiB
    member = oracle.gzip_compress(data)
    assert member == _zlib_gzip_member(data)
    assert gzip.decompress(member) == data


def test_deflate_full_c2_row_group_pages():
    """Every page of one whole C2 row group (Rec8, seed 0xC0FFEE02, the reference's 128 MiB row
    groups and pages: the first row group holds 2.08 M records, 50.7 MB of page bytes, its PLAIN
    int64 pages 16.6 MB each, deflate's window sliding ~500 times per page) deflated by the
    oracle, byte-identical to zlib's level-6 member.  The pages the GZIP writer compresses are
    the UNCOMPRESSED file's page bodies (at pageSize = blockSize nothing is flushed before a cut,
    so the codec moves no cut)."""
    data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE02, 2_300_000)
    fb = oracle.encode_file(synth.REC8, data, offs, oracle.make_props(codec=oracle.UNCOMPRESSED))
    del data, offs
    pages = [pg["body"] for pg in pqwalk.pages(fb) if pg["rg"] == 0]
    assert sum(len(b) for b in pages) > 48 * MiB and max(len(b) for b in pages) > 16 * 10 ** 6
    assert any(pg["rg"] == 1 for pg in pqwalk.pages(fb))   # row group 0 is complete (cut before the end)
    for body in pages:
        assert oracle.gzip_compress(body) == _zlib_gzip_member(body)


def _readback(schema, recs, fb):
    tbl = pq.read_table(io.BytesIO(fb))
    assert tbl.num_rows == len(recs)
    assert protoutil.table_columns(tbl, schema) == protoutil.decode_columns(schema, recs)


CASES = [
    (synth.KIND_SAMPLE, 0, 3000), (synth.KIND_SAMPLE, 30, 3000),
    (synth.KIND_REC8, 0, 5000), (synth.KIND_HIGHCARD, 0, 1500),
]


CODEC_NAMES = {oracle.UNCOMPRESSED: "none", oracle.SNAPPY: "snappy", oracle.GZIP: "gzip"}


@pytest.mark.parametrize("kind,param,n", CASES)
@pytest.mark.parametrize("codec", [oracle.UNCOMPRESSED, oracle.SNAPPY, oracle.GZIP])
@pytest.mark.parametrize("page_size,block_size", [(128 * MiB, 128 * MiB), (MiB, 128 * MiB), (8192, 64 * 1024)])
@pytest.mark.parametrize("dictionary", [True, False])
def test_oracle_readback(kind, param, n, codec, page_size, block_size, dictionary):
    schema = synth.SCHEMAS[kind]
    data, offs = synth.generate(kind, 0xC0FFEE01 + kind, n, param=param)
    props = oracle.make_props(block_size=block_size, page_size=page_size, codec=codec, enable_dictionary=dictionary)
    fb = oracle.encode_file(schema, data, offs, props)
    _readback(schema, synth.records(data, offs), fb)
    # every page decodes with an independent Snappy / gzip, header sizes consistent
    for pg, raw in pqwalk.decompress_pages(fb, CODEC_NAMES[codec]):
        if codec == oracle.GZIP:   # and is exactly zlib's member of the uncompressed page
            assert pg["body"] == _zlib_gzip_member(raw)


V2_CASES = [(synth.KIND_SAMPLE, 30, 3000), (synth.KIND_REC8, 0, 4000), (synth.KIND_HIGHCARD, 0, 1500)]


@pytest.mark.parametrize("kind,param,n", V2_CASES)
@pytest.mark.parametrize("codec", [oracle.UNCOMPRESSED, oracle.SNAPPY, oracle.GZIP])
@pytest.mark.parametrize("page_size,block_size", [(128 * MiB, 128 * MiB), (8192, 64 * 1024)])
@pytest.mark.parametrize("dictionary", [True, False])
def test_oracle_v2_readback(kind, param, n, codec, page_size, block_size, dictionary):
    """PARQUET_2_0 (A10): DataPageV2, RLE_DICTIONARY, DELTA_BINARY_PACKED / DELTA_BYTE_ARRAY
    fallback, RLE booleans — every file reads back value-exact through pyarrow."""
    schema = synth.SCHEMAS[kind]
    data, offs = synth.generate(kind, 0xC0FFEE11 + kind, n, param=param)
    props = oracle.make_props(block_size=block_size, page_size=page_size, codec=codec, enable_dictionary=dictionary,
                              writer_version=2)
    fb = oracle.encode_file(schema, data, offs, props)
    _readback(schema, synth.records(data, offs), fb)
    pqwalk.decompress_pages(fb, CODEC_NAMES[codec])
    assert {p["header"][1] for p in pqwalk.pages(fb)} <= {2, 3}   # dictionary + DataPageV2 only


def _arrow_v2_values(arr, encoding):
    """Values bytes of the single DataPageV2 pyarrow writes for a non-nullable column."""
    t = pa.table({"x": arr}, schema=pa.schema([pa.field("x", arr.type, nullable=False)]))
    b = io.BytesIO()
    pq.write_table(t, b, use_dictionary=False, column_encoding={"x": encoding}, data_page_version="2.0",
                   compression="NONE", write_statistics=False)
    pgs = [p for p in pqwalk.pages(b.getvalue()) if p["header"][1] == 3]
    assert len(pgs) == 1
    h = pgs[0]["header"][8]
    return pgs[0]["body"][h[5] + h[6]:]


@pytest.mark.parametrize("n", [1, 2, 33, 100, 129, 257, 1 + 128 * 40])
@pytest.mark.parametrize("kind", ["small", "wide", "neg", "const"])
def test_delta_int32_matches_pyarrow(n, kind):
    """DeltaBinaryPackingValuesWriterForInteger vs Arrow's independent DELTA_BINARY_PACKED
    encoder (same 128-value blocks / 4 miniblocks for int32): byte-identical whenever the
    page has no partial block after a full one — the only place parquet-mr's never-cleared
    bitWidths/deltaBlockBuffer show (pinned separately below)."""
    rng = np.random.default_rng(n * 7 + len(kind))
    if kind == "small":
        v = np.cumsum(rng.integers(-5, 50, n))
    elif kind == "wide":
        v = rng.integers(-2 ** 31, 2 ** 31, n)
    elif kind == "neg":
        v = -np.arange(n) * 7
    else:
        v = np.full(n, 42)
    v = v.astype(np.int32)
    assert oracle.delta_encode(v.astype(np.int64), False) == _arrow_v2_values(pa.array(v, type=pa.int32()),
                                                                           "DELTA_BINARY_PACKED")


def test_delta_partial_block_stale_state():
    """parquet-mr quirk restated: a partial last block writes the previous block's widths for
    its missing miniblocks and packs the previous block's reduced deltas as padding (Arrow
    writes zeros there).  Everything before the last block's width bytes is identical."""
    def varint_at(b, p):
        r = s = 0
        while True:
            c = b[p]
            p += 1
            r |= (c & 0x7F) << s
            s += 7
            if not c & 0x80:
                return r, p

    v = np.cumsum(np.random.default_rng(5).integers(0, 1000, 200)).astype(np.int32)   # 128 + 71 deltas
    ours = oracle.delta_encode(v.astype(np.int64), False)
    arrow = _arrow_v2_values(pa.array(v, type=pa.int32()), "DELTA_BINARY_PACKED")
    assert len(ours) == len(arrow) and ours != arrow
    p = 0
    for _ in range(4):                       # block size, miniblocks, count, first value
        _, p = varint_at(ours, p)
    _, p = varint_at(ours, p)                # block 0: min delta
    w0 = list(ours[p:p + 4])
    p += 4 + sum(4 * w for w in w0)
    _, p = varint_at(ours, p)                # block 1: min delta
    w1 = list(ours[p:p + 4])
    assert ours[:p + 3] == arrow[:p + 3]     # identical up to the first stale width byte
    assert w1[3] == w0[3] and arrow[p + 3] == 0   # 3 miniblocks present; the 4th width is block 0's
    pad0 = p + 4 + 4 * w1[0] + 4 * w1[1] + (7 * w1[2] + 7) // 8   # 7 real values in miniblock 2
    assert ours[p + 4:pad0 - 1] == arrow[p + 4:pad0 - 1]
    assert any(ours[pad0:]) and not any(arrow[pad0:])   # stale padding vs zeros


@pytest.mark.parametrize("n", [1, 5, 129, 257, 1 + 128 * 9])
def test_delta_byte_array_matches_pyarrow(n):
    """DeltaByteArrayWriter (prefix lengths + DeltaLengthByteArray suffixes) vs Arrow's
    DELTA_BYTE_ARRAY encoder, through a whole v2 file of the oracle (no dictionary)."""
    rng = np.random.default_rng(n)
    words = [("key%04d" % int(rng.integers(0, 300))).encode() +
             bytes(rng.integers(97, 100, int(rng.integers(0, 6))).astype(np.uint8)) for _ in range(n)]
    recs = [b"\x0a" + _varint(len(w)) + w + b"\x10" + _varint(i) for i, w in enumerate(words)]
    data, offs = synth.pack(recs)
    fb = oracle.encode_file(synth.SAMPLE, data, offs, oracle.make_props(writer_version=2, enable_dictionary=False))
    page = [p for p in pqwalk.pages(fb) if p["col"] == 0][0]
    h = page["header"][8]
    # the width-0 level streams of this REQUIRED column (ColumnWriterV2 level encoders) come first
    assert (h[5], h[6]) == ((1, 1) if n < 8 else (len(_varint(n << 1)),) * 2)
    assert page["body"][h[5] + h[6]:] == _arrow_v2_values(pa.array(words, type=pa.binary()), "DELTA_BYTE_ARRAY")


def _sample_msg(**kw):
    return wire_cases.sample_msg(**kw)


_varint = wire_cases.varint


def test_proto_edge_cases_accepted():
    """Unknown fields skipped, last occurrence wins, any field order, 10-byte negative
    int32, unknown groups, known number with a foreign wire type treated as unknown
    (protobuf-java generated switch-on-tag; TestMessage.java:85-139).  The same records go
    through the HIP decoder in test_gpu_wire.py."""
    recs = [r for _, r in wire_cases.accepted()]
    data, offs = synth.pack(recs)
    fb = oracle.encode_file(synth.SAMPLE, data, offs)
    _readback(synth.SAMPLE, recs, fb)


@pytest.mark.parametrize("label,bad", wire_cases.invalid(), ids=[c[0] for c in wire_cases.invalid()])
def test_proto_invalid_rejected(label, bad):
    w = oracle.OracleWriter(synth.SAMPLE)
    good = _sample_msg(query="x", timestamp=1).SerializeToString()
    w.write(good)
    with pytest.raises(oracle.OracleError) as e:
        w.write(bad)
    assert e.value.status == -3
    assert w.num_records() == 1
    w.close()
    _readback(synth.SAMPLE, [good], w.file_bytes())
    # google.protobuf's own parser rejects it too (the reference's parseFrom would throw)
    cls = protoutil.message_class(synth.SAMPLE)
    with pytest.raises(Exception):
        m = cls.FromString(bad)
        if not m.IsInitialized():
            raise ValueError("missing required")


DESC = json.load(open(os.path.join(HERE, "golden", "test_message_descriptor.json")))


def _kv(fb):
    return {kv[1].decode(): kv[2].decode() for kv in pqwalk.footer(fb)[5]}


def test_descriptor_fixture_matches_sample_schema():
    """The schema the tests use for the reference's test message equals the descriptor the
    reference itself holds (TestMessage.java:750-755 descriptorData, decoded into
    tests/golden/test_message_descriptor.json by make_descriptor_fixture.py)."""
    from google.protobuf import descriptor_pb2
    fdp = descriptor_pb2.FileDescriptorProto.FromString(bytes.fromhex(DESC["file_descriptor_hex"]))
    assert [[f.name, f.number, f.type, f.label] for f in fdp.message_type[0].field] == DESC["columns"]
    assert [list(c) for c in synth.SAMPLE.columns] == DESC["columns"]
    assert synth.SAMPLE.message_name == DESC["message_full_name"]
    assert synth.SAMPLE.proto_class == DESC["proto_class"]


def test_footer_pinned_to_reference_descriptor():
    """ProtoWriteSupport.init's extra metadata (parquet-protobuf 1.10.1): parquet.proto.class
    = the message class, parquet.proto.descriptor = TextFormat of descriptor.toProto();
    ProtoSchemaConverter: schema name = full name, one REQUIRED/OPTIONAL leaf per field with
    field_id = field number, strings as BINARY/UTF8."""
    data, offs = synth.generate(synth.KIND_SAMPLE, 3, 200)
    fb = oracle.encode_file(synth.SAMPLE, data, offs)
    kv = _kv(fb)
    assert kv["parquet.proto.descriptor"] == DESC["descriptor_text"]
    assert kv["parquet.proto.class"] == DESC["proto_class"]
    assert kv["writer.model.name"] == "protobuf"
    schema = pqwalk.footer(fb)[2]
    assert schema[0][4].decode() == DESC["message_full_name"] and schema[0][5] == len(DESC["columns"])
    phys = {9: 6, 3: 2, 5: 1}   # TYPE_STRING -> BYTE_ARRAY, TYPE_INT64 -> INT64, TYPE_INT32 -> INT32
    for el, (name, number, ptype, label) in zip(schema[1:], DESC["columns"]):
        assert el[4].decode() == name and el[9] == number and el[1] == phys[ptype]
        assert el[3] == (0 if label == 2 else 1)            # REQUIRED / OPTIONAL
        assert (el.get(6) == 0) == (ptype == 9)             # ConvertedType UTF8 for strings


def _chunk_encodings(fb):
    fm = pqwalk.footer(fb)
    return [[cc[3][2] for cc in rg[1]] for rg in fm[4]]


def test_dictionary_fallback_and_satisfying():
    # HIGHCARD: uuid/blob exceed 1 MiB of dictionary -> PLAIN; code (<=1000 values) stays dictionary
    data, offs = synth.generate(synth.KIND_HIGHCARD, 5, 40000)
    fb = oracle.encode_file(synth.HIGHCARD, data, offs, oracle.make_props(codec=oracle.SNAPPY))
    enc = _chunk_encodings(fb)[0]
    assert 2 not in enc[1] and 2 not in enc[2]  # uuid, blob: no PLAIN_DICTIONARY
    assert 2 in enc[3]                           # code: PLAIN_DICTIONARY
    # dictionary page only where the dictionary was used
    kinds = [(p["col"], p["header"][1]) for p in pqwalk.pages(fb)]
    assert (3, 2) in kinds and (1, 2) not in kinds and (2, 2) not in kinds


def test_all_null_first_page_falls_back():
    # every optional value null: the first page's bit width is 32, isCompressionSatisfying
    # fails (1 byte vs 0 raw) and the chunk is PLAIN with no dictionary page.
    recs = [_sample_msg(query="q%d" % (i % 3), timestamp=i).SerializeToString() for i in range(500)]
    data, offs = synth.pack(recs)
    fb = oracle.encode_file(synth.SAMPLE, data, offs)
    enc = _chunk_encodings(fb)[0]
    assert 2 not in enc[2] and 2 not in enc[3]
    _readback(synth.SAMPLE, recs, fb)


def test_max_file_size_rotation():
    """KafkaProtoParquetWriterTest.testMaxFileSize restated (:142-174): 10 KiB row groups,
    maxFileSize 100 KiB, the WorkerThread closes a file right after the record that makes
    getDataSize() >= maxFileSize (KPW:281-285,306-308); every closed file satisfies
    0.9 < maxFileSize/len < 1.01."""
    max_file = 100 * 1024
    props = oracle.make_props(block_size=10 * 1024)
    data, offs = synth.generate(synth.KIND_SAMPLE, 0xC0FFEE01, 6000)
    files, start = [], 0
    while len(files) < 2:
        w = oracle.OracleWriter(synth.SAMPLE, props)
        sub = offs[start:] - offs[start]
        st, na, full = w.write_until_full(data[int(offs[start]):], sub, max_file)
        assert st == 0
        if not full:
            break
        w.close()
        files.append(w.file_bytes())
        start += na
    assert len(files) >= 2
    for fb in files:
        r = max_file / len(fb)
        assert 0.9 < r < 1.01, r
        assert pq.read_table(io.BytesIO(fb)).num_rows > 0


def test_round_trip_multiset_sample():
    """testMaxOpenDuration's containsInAnyOrder check restated (:136-139)."""
    data, offs = synth.generate(synth.KIND_SAMPLE, 77, 100)
    recs = synth.records(data, offs)
    fb = oracle.encode_file(synth.SAMPLE, data, offs)
    cls = protoutil.message_class(synth.SAMPLE)
    tbl = pq.read_table(io.BytesIO(fb)).to_pylist()
    got = sorted(cls(**{k: v for k, v in row.items() if v is not None}).SerializeToString() for row in tbl)
    want = sorted(cls.FromString(r).SerializeToString() for r in recs)
    assert got == want


def test_get_data_size_tracks_file():
    data, offs = synth.generate(synth.KIND_REC8, 3, 20000)
    w = oracle.OracleWriter(synth.REC8, oracle.make_props(block_size=256 * 1024))
    last = 0
    for i in range(0, 20000, 1000):
        st, nw = w.write_batch(data, offs[i:i + 1001])
        assert st == 0
        ds = w.data_size()
        assert ds > 0
        last = ds
    assert w.num_row_groups() >= 2
    w.close()
    fb = w.file_bytes()
    assert abs(len(fb) - last) < 0.2 * len(fb)


@pytest.mark.parametrize("kind,n", [(synth.KIND_REC8, 300_000), (synth.KIND_WIDE, 20_000), (synth.KIND_HIGHCARD, 60_000)])
def test_row_groups_are_independent(kind, n):
    """The premise of tests/test_gpu_fullsize.py: a whole-file oracle encode equals, row group
    by row group, the oracle re-run from each row group's first record (cut re-derived from
    [start, end + 10001), chunk bytes and metadata identical)."""
    from gpu_helpers import check_row_groups
    schema = synth.SCHEMAS[kind]
    data, offs = synth.generate(kind, 0xC0FFEE00 + kind, n)
    props = oracle.make_props(block_size=1024 * 1024, codec=1)
    fb = oracle.encode_file(schema, data, offs, props)
    import pqwalk
    assert len(pqwalk.footer(fb)[4]) > 3
    assert check_row_groups(schema, data, offs, fb, props) == []
    # and it does see a changed byte: the first page body byte of the last row group's chunk 0
    last = [pg for pg in pqwalk.pages(fb) if pg["col"] == 0][-1]
    bad = bytearray(fb)
    body_at = fb.index(last["body"], last["offset"])
    bad[body_at] ^= 0x01
    errs = check_row_groups(schema, data, offs, bytes(bad), props)
    assert errs and "chunk bytes differ" in errs[0]
