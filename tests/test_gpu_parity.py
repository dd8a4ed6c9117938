"""GPU parity: pages from the HIP path (through the C-ABI) byte-identical to the CPU oracle.

Bar: bit-exact (integer/byte work).  Sizes are small enough for the oracle to finish in
seconds; the full-size bench workload is checked by size-independent properties in
test_gpu_properties.py.
"""
import io

import numpy as np
import pyarrow.parquet as pq
import pytest

import gpu_helpers as gh
import oracle
import protoutil
import synth

pytestmark = pytest.mark.gpu
MiB = 1024 * 1024

CASES = [
    ("sample", synth.KIND_SAMPLE, 0, 3000),
    ("sample_nulls", synth.KIND_SAMPLE, 30, 3000),
    ("rec8", synth.KIND_REC8, 0, 20000),
    ("highcard", synth.KIND_HIGHCARD, 0, 4000),
    ("wide", synth.KIND_WIDE, 0, 600),
]


@pytest.mark.parametrize("name,kind,param,n", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("codec", [0, 1, 2], ids=["uncompressed", "snappy", "gzip"])
@pytest.mark.parametrize("block_size", [128 * MiB, 64 * 1024], ids=["rg128M", "rg64K"])
def test_pages_match_oracle(name, kind, param, n, codec, block_size):
    schema = synth.SCHEMAS[kind]
    data, offs = synth.generate(kind, 0xC0FFEE01 + kind, n, param=param)
    errs = gh.compare_pages(schema, data, offs, codec=codec, block_size=block_size)
    assert not errs, "\n".join(errs[:12])


@pytest.mark.parametrize("name,kind,param,n", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("codec", [0, 1, 2], ids=["uncompressed", "snappy", "gzip"])
@pytest.mark.parametrize("block_size", [128 * MiB, 64 * 1024], ids=["rg128M", "rg64K"])
def test_v2_pages_match_oracle(name, kind, param, n, codec, block_size):
    """A10 / PARQUET_2_0: DataPageV2 headers, unprefixed levels in front of the compressed
    values, RLE_DICTIONARY, RLE booleans (their RLE bytes in the row-group size check),
    DELTA_BINARY_PACKED / DELTA_BYTE_ARRAY fallback pages byte-identical to the oracle."""
    schema = synth.SCHEMAS[kind]
    data, offs = synth.generate(kind, 0xC0FFEE21 + kind, n, param=param)
    errs = gh.compare_pages(schema, data, offs, codec=codec, block_size=block_size, writer_version=2)
    assert not errs, "\n".join(errs[:12])


@pytest.mark.parametrize("kind,n", [(synth.KIND_HIGHCARD, 40000), (synth.KIND_REC8, 300000)], ids=["highcard", "rec8"])
def test_v2_delta_fallback_large(kind, n):
    # uuid/blob fall back to DELTA_BYTE_ARRAY, ts/user_id to DELTA_BINARY_PACKED (many 128-value
    # blocks, partial last blocks with parquet-mr's stale widths and padding)
    import pqwalk
    schema = synth.SCHEMAS[kind]
    data, offs = synth.generate(kind, 5, n)
    errs = gh.compare_pages(schema, data, offs, codec=1, writer_version=2)
    assert not errs, "\n".join(errs[:12])
    fb = oracle.encode_file(schema, data, offs, oracle.make_props(codec=1, writer_version=2))
    encs = {p["header"][8][4] for p in pqwalk.pages(fb) if p["header"][1] == 3}
    # highcard: uuid/blob DELTA_BYTE_ARRAY; rec8: ts/user_id DELTA_BINARY_PACKED, price PLAIN
    assert (7 in encs) if kind == synth.KIND_HIGHCARD else (5 in encs and 0 in encs), encs


@pytest.mark.parametrize("n", [1, 2, 3, 33, 128, 129, 130, 257, 1000])
def test_v2_delta_block_edges(n):
    """Stream lengths around the 128-value block and 32-value miniblock boundaries; the
    dictionary is forced off by its compression check (all-distinct timestamps/queries)."""
    cls = protoutil.message_class(synth.SAMPLE)
    recs = [cls(query="q%07d" % (i * 7919 % 1000003), timestamp=(i * 2654435761) % (1 << 40) - (1 << 39),
                page_number=(-i if i % 3 else i)).SerializeToString() for i in range(n)]
    data, offs = synth.pack(recs)
    for codec in (0, 1):
        errs = gh.compare_pages(synth.SAMPLE, data, offs, codec=codec, writer_version=2)
        assert not errs, "\n".join(errs[:12])


def test_v2_writer_file_identical():
    import kpw
    import pqwalk
    schema = synth.REC8
    data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE31, 20000, param=0)
    props = kpw.ParquetProperties(block_size=256 * 1024, compression_codec_name=1, writer_version=2)
    fb = gh.gpu_file(schema, data, offs, props, batches=3)
    ob = oracle.encode_file(schema, data, offs, oracle.make_props(block_size=256 * 1024, codec=1, writer_version=2))
    assert fb == ob, pqwalk.first_difference(fb, ob)
    tbl = pq.read_table(io.BytesIO(fb))
    assert protoutil.table_columns(tbl, schema) == protoutil.decode_columns(schema, synth.records(data, offs))


@pytest.mark.parametrize("dictionary", [True, False])
def test_dictionary_toggle(dictionary):
    data, offs = synth.generate(synth.KIND_REC8, 11, 5000)
    errs = gh.compare_pages(synth.REC8, data, offs, codec=1, dictionary=dictionary)
    assert not errs, "\n".join(errs[:12])


def test_fallback_highcard_large():
    # uuid/blob exceed the 1 MiB dictionary: PLAIN; code keeps PLAIN_DICTIONARY
    data, offs = synth.generate(synth.KIND_HIGHCARD, 5, 40000)
    errs = gh.compare_pages(synth.HIGHCARD, data, offs, codec=1)
    assert not errs, "\n".join(errs[:12])


@pytest.mark.parametrize("kind,n,block_size", [(synth.KIND_REC8, 400_000, 2 * MiB),
                                               (synth.KIND_REC8, 700_000, 12 * MiB),
                                               (synth.KIND_SAMPLE, 300_000, 3 * MiB)],
                         ids=["rec8_2MiB", "rec8_12MiB", "sample_3MiB"])
def test_planner_clamp_regime(kind, n, block_size):
    # row groups of ~10^5 records: most checks take the recordCount + 10000 clamp, which the
    # planner evaluates 64 check points at a time once the def-level walkers converge
    schema = synth.SCHEMAS[kind]
    data, offs = synth.generate(kind, 0xC0FFEE07, n, param=20)
    errs = gh.compare_pages(schema, data, offs, codec=1, block_size=block_size)
    assert not errs, "\n".join(errs[:12])


def test_edge_cases():
    cls = protoutil.message_class(synth.SAMPLE)
    recs = []
    for i in range(700):  # long all-null run, then alternation, then all-present
        m = cls(query="q%d" % (i % 7), timestamp=i)
        if 300 <= i < 500 and i % 2:
            m.page_number = -i
        if i >= 500:
            m.page_number = i % 3
            m.result_per_page = 5
        recs.append(m.SerializeToString())
    data, offs = synth.pack(recs)
    for codec in (0, 1):
        errs = gh.compare_pages(synth.SAMPLE, data, offs, codec=codec)
        assert not errs, "\n".join(errs[:12])


def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _snappy_strings(pattern, rng):
    """Query strings whose PLAIN page stresses one Snappy regime (multi-fragment pages)."""
    out = []
    if pattern == "random":          # incompressible: long literal searches, skip growth
        for _ in range(1500):
            out.append(rng.integers(0, 256, int(rng.integers(0, 400)), dtype=np.uint8).tobytes())
    elif pattern == "periodic":      # short periods: back-to-back matches, table churn
        for i in range(2500):
            p = 1 + i % 37
            unit = rng.integers(0, 256, p, dtype=np.uint8).tobytes()
            out.append((unit * (200 // p + 1))[: int(rng.integers(1, 200))])
    elif pattern == "zeros":         # long runs: copies split at 64/68 bytes
        for i in range(600):
            out.append(bytes(int(rng.integers(0, 2000))))
    elif pattern == "nearrep":       # copies of earlier strings with point mutations
        base = [rng.integers(0, 256, 60, dtype=np.uint8).tobytes() for _ in range(40)]
        for i in range(4000):
            b = bytearray(base[int(rng.integers(0, 40))])
            for _ in range(int(rng.integers(0, 4))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            out.append(bytes(b[: int(rng.integers(4, 61))]))
    elif pattern == "mixed":         # alternating regimes inside one fragment
        for i in range(3000):
            k = i % 4
            if k == 0:
                out.append(rng.integers(0, 256, int(rng.integers(0, 90)), dtype=np.uint8).tobytes())
            elif k == 1:
                out.append(b"abcd" * int(rng.integers(0, 30)))
            elif k == 2:
                out.append(bytes([int(rng.integers(0, 4))]) * int(rng.integers(0, 50)))
            else:
                out.append(("%08d" % int(rng.integers(0, 10 ** 8))).encode() * 3)
    elif pattern == "tiny":          # pages shorter than snappy's 15-byte input margin
        out = [b"", b"x"]
    return out


@pytest.mark.parametrize("pattern", ["random", "periodic", "zeros", "nearrep", "mixed", "tiny"])
def test_snappy_patterns(pattern):
    # dictionary off so the query page is the raw PLAIN strings (the K7 input as written)
    rng = np.random.default_rng(sum(pattern.encode()))
    recs = [b"\x0a" + _varint(len(q)) + q + b"\x10" + _varint(i) for i, q in enumerate(_snappy_strings(pattern, rng))]
    data, offs = synth.pack(recs)
    errs = gh.compare_pages(synth.SAMPLE, data, offs, codec=1, dictionary=False)
    assert not errs, "\n".join(errs[:12])


_TRICKY = [b"", b"\x00", b"a", b"a\x00", b"a\x00\x00", b"ab" * 8, b"ab" * 8 + b"\x00", b"ab" * 8 + b"\x01",
           b"ab" * 8 + b"\x00\x00", b"ab" * 10, b"ab" * 10 + b"c", b"ab" * 9 + b"a", b"\xff" * 16, b"\xff" * 17,
           b"\xff" * 15 + b"\xfe", b"\x7f" * 20, b"\x80" + b"\x00" * 30, b"\x80" + b"\x00" * 31, b"zz", b"z" * 40]


@pytest.mark.parametrize("dictionary", [True, False], ids=["entries", "values"])
@pytest.mark.parametrize("subset", ["all", "no_extremes"])
def test_string_stats_tricky(dictionary, subset):
    # BYTE_ARRAY min/max (unsigned lexicographic, shorter first) through the 16-byte prefix
    # arrays: ties on the prefix, embedded zeros, lengths 0/16/17, high bytes
    pool = _TRICKY if subset == "all" else [q for q in _TRICKY if q not in (b"", b"\xff" * 17, b"z" * 40)]
    rng = np.random.default_rng(7 if dictionary else 8)
    recs = []
    for i in range(5000):
        q = pool[int(rng.integers(0, len(pool)))]
        recs.append(b"\x0a" + _varint(len(q)) + q + b"\x10" + _varint(i))
    data, offs = synth.pack(recs)
    for codec in (0, 1):
        errs = gh.compare_pages(synth.SAMPLE, data, offs, codec=codec, dictionary=dictionary)
        assert not errs, "\n".join(errs[:12])


@pytest.mark.parametrize("n", [1, 7, 8, 9, 63, 64, 65, 100, 101, 255])
def test_tiny_batches(n):
    data, offs = synth.generate(synth.KIND_REC8, 99, n)
    errs = gh.compare_pages(synth.REC8, data, offs, codec=1, block_size=4096)
    assert not errs, "\n".join(errs[:12])


@pytest.mark.parametrize("kind", [synth.KIND_SAMPLE, synth.KIND_REC8])
@pytest.mark.parametrize("codec", [0, 1, 2], ids=["uncompressed", "snappy", "gzip"])
@pytest.mark.parametrize("n,batches", [(20000, 3), (300000, 2)], ids=["model", "bulk"])
def test_writer_file_identical(kind, codec, n, batches):
    """The ParquetFile drop-in writes the same file bytes as the oracle, across several
    write batches: small batches go through the host size model (row groups cut on the host),
    batches of > 65536 records through the GPU planner (open row groups carried between jobs)."""
    schema = synth.SCHEMAS[kind]
    data, offs = synth.generate(kind, 0xC0FFEE01, n)
    import kpw
    props = kpw.ParquetProperties(block_size=256 * 1024, compression_codec_name=codec)
    fb = gh.gpu_file(schema, data, offs, props, batches=batches)
    ob = oracle.encode_file(schema, data, offs, oracle.make_props(block_size=256 * 1024, codec=codec))
    import pqwalk
    assert fb == ob, pqwalk.first_difference(fb, ob)
    tbl = pq.read_table(io.BytesIO(fb))
    assert protoutil.table_columns(tbl, schema) == protoutil.decode_columns(schema, synth.records(data, offs))


def test_invalid_record_cuts_batch():
    """Small write (size-model path): the write itself raises at the invalid record, like the
    reference's parseFrom (KafkaProtoParquetWriter.java:270-276)."""
    import kpw
    good = synth.records(*synth.generate(synth.KIND_SAMPLE, 1, 50))
    bad = b"\x10\x01"  # missing required query
    pf = kpw.ParquetFile(None, kpw.Schema(synth.SAMPLE.message_name, synth.SAMPLE.columns))
    with pytest.raises(kpw.InvalidProtoError) as e:
        pf.write_batch(good + [bad] + good[:5])
    assert e.value.record == 50
    assert pf.get_num_written_records() == 50
    with pytest.raises(kpw.InvalidProtoError):
        pf.get_data_size()
    pf.close()
    tbl = pq.read_table(io.BytesIO(pf.file_bytes()))
    assert tbl.num_rows == 50


@pytest.mark.gpu
@pytest.mark.parametrize("codec", [0, 1])
@pytest.mark.parametrize("n,batches", [(60000, 40), (400000, 2)], ids=["model", "bulk"])
@pytest.mark.parametrize("dfs,pad", [(384 * 1024, 96 * 1024), (300 * 1024, 32 * 1024), (256 * 1024, 64 * 1024)],
                         ids=["dfs1.5x", "dfs-odd", "dfs=block"])
def test_writer_hdfs_alignment(codec, n, batches, dfs, pad):
    """HDFS PaddingAlignment (ParquetFileWriter 1.10.1; the reference's target file system,
    KafkaProtoParquetWriter.java:137-141): row-group limits follow the HDFS block position of
    the previous row group's end, zero padding fills a block tail <= maxPaddingSize.  Many row
    groups cross many dfs blocks; file bytes identical to the oracle (oracle_core.c
    align_for_row_group / next_row_group_size), on the size-model and bulk paths."""
    import kpw
    schema = synth.REC8
    data, offs = synth.generate(synth.KIND_REC8, 0xD15C, n)
    props = kpw.ParquetProperties(block_size=256 * 1024, compression_codec_name=codec, dfs_block_size=dfs,
                                  max_padding_size=pad)
    fb = gh.gpu_file(schema, data, offs, props, batches=batches)
    ob = oracle.encode_file(schema, data, offs, oracle.make_props(block_size=256 * 1024, codec=codec,
                                                                   dfs_block_size=dfs, max_padding_size=pad))
    import pqwalk
    assert fb == ob, pqwalk.first_difference(fb, ob)
    fm = pqwalk.footer(fb)
    assert len(fm[4]) >= 8
    tbl = pq.read_table(io.BytesIO(fb))
    assert tbl.num_rows == n


@pytest.mark.gpu
def test_writer_hdfs_data_size_every_record():
    """getDataSize after every record with HDFS alignment (host size model with the per-row-group
    limit) equals the oracle's on every record, and the file is identical."""
    import kpw
    schema = synth.SAMPLE
    data, offs = synth.generate(synth.KIND_SAMPLE, 0xA11C, 30000)
    recs = synth.records(data, offs)
    props = kpw.ParquetProperties(block_size=64 * 1024, dfs_block_size=100 * 1024, max_padding_size=16 * 1024)
    pf = kpw.ParquetFile(None, kpw.Schema(schema.message_name, schema.columns, schema.proto_class), props)
    ow = oracle.OracleWriter(schema, oracle.make_props(block_size=64 * 1024, dfs_block_size=100 * 1024,
                                                       max_padding_size=16 * 1024))
    bad = []
    for i, r in enumerate(recs):
        pf.write(r)
        ow.write(r)
        a, b = pf.get_data_size(), ow.data_size()
        if a != b:
            bad.append((i, a, b))
            if len(bad) > 5:
                break
    assert not bad, bad
    pf.close()
    ow.close()
    assert pf.file_bytes() == ow.file_bytes()


@pytest.mark.gpu
@pytest.mark.parametrize("codec", [0, 1])
def test_writer_hdfs_alignment_multipage(codec):
    """HDFS alignment with multi-page chunks (pageSize < blockSize: the row-group limit is
    checked against flushed pages' compressed bytes) — identical file bytes."""
    import kpw
    schema = synth.REC8
    n = 250000
    data, offs = synth.generate(synth.KIND_REC8, 0x3A6E, n)
    kw = dict(block_size=512 * 1024, dfs_block_size=700 * 1024, max_padding_size=100 * 1024)
    props = kpw.ParquetProperties(compression_codec_name=codec, page_size=64 * 1024, **kw)
    fb = gh.gpu_file(schema, data, offs, props, batches=3)
    ob = oracle.encode_file(schema, data, offs, oracle.make_props(codec=codec, page_size=64 * 1024, **kw))
    import pqwalk
    assert fb == ob, pqwalk.first_difference(fb, ob)
    assert len(pqwalk.footer(fb)[4]) >= 4


@pytest.mark.parametrize("n,batches", [(20000, 3), (300000, 2)], ids=["model", "bulk"])
def test_writer_local_file_identical(tmp_path, n, batches):
    """File mode (a path instead of an in-memory file: pages D2H to pinned staging, fwrite on the
    assembly thread) writes the same bytes as the oracle."""
    import kpw
    schema = synth.REC8
    data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE07, n)
    props = kpw.ParquetProperties(block_size=256 * 1024, compression_codec_name=1)
    path = str(tmp_path / "part-0.parquet")
    pf = kpw.ParquetFile(path, kpw.Schema(schema.message_name, schema.columns, schema.proto_class), props)
    step = (n + batches - 1) // batches
    for i in range(0, n, step):
        j = min(n, i + step)
        pf.write_batch((data[int(offs[i]):int(offs[j])], offs[i:j + 1] - offs[i]))
    pf.close()
    fb = open(path, "rb").read()
    ob = oracle.encode_file(schema, data, offs, oracle.make_props(block_size=256 * 1024, codec=1))
    import pqwalk
    assert fb == ob, pqwalk.first_difference(fb, ob)


def _card_batch(n, card, seed):
    """SampleMessage records whose four columns each take `card` distinct values."""
    rng = np.random.default_rng(seed)
    k = rng.integers(0, card, n)
    recs = []
    for i in range(n):
        v = int(k[i])
        q = b"k%09d" % v
        rec = b"\x0a" + _varint(len(q)) + q + b"\x10" + _varint(1_700_000_000_000 + v)
        if i % 5:
            rec += b"\x18" + _varint(v)
        if i % 3:
            rec += b"\x20" + _varint((v * 7) % card)
        recs.append(rec)
    return synth.pack(recs)


def test_dictionary_table_hints_across_encodes():
    """One encoder over batches whose cardinality jumps: each encode sizes its dictionary hash
    tables from the previous one's entry counts (engine.cpp assign_tables); a table that turns
    out too small is redone at full size.  Every batch must stay byte-identical to the oracle
    (including a jump past the 1 MiB dictionary fallback)."""
    import kpw
    enc = kpw.Encoder(kpw.Schema(synth.SAMPLE.message_name, synth.SAMPLE.columns, synth.SAMPLE.proto_class), codec=1,
                      block_size=128 * gh.MiB, page_size=128 * gh.MiB, enable_dictionary=True, writer_version=1)
    for j, card in enumerate((40, 30000, 40, 150000, 3000)):
        data, offs = _card_batch(200_000, card, 77 + j)
        fb = oracle.encode_file(synth.SAMPLE, data, offs, gh.oracle_props(codec=1))
        errs, _ = gh.compare_to_file(synth.SAMPLE, data, offs, fb, codec=1, enc=enc)
        assert not errs, ("batch %d (card %d): " % (j, card)) + "\n".join(errs[:12])


_SPLIT_CHILD = r"""
import sys
sys.path[:0] = sys.argv[1].split(":")
import kpw, oracle, pqwalk, synth
schema = synth.REC8
n = 2_400_000
data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE09, n)
props = kpw.ParquetProperties(block_size=1 << 20, compression_codec_name=1)
pf = kpw.ParquetFile(None, kpw.Schema(schema.message_name, schema.columns, schema.proto_class), props)
for i in range(0, n, 1_200_000):
    j = min(n, i + 1_200_000)
    pf.write_batch((data[int(offs[i]):int(offs[j])], offs[i:j + 1] - offs[i]))
pf.close()
fb = pf.file_bytes()
ob = oracle.encode_file(schema, data, offs, oracle.make_props(block_size=1 << 20, codec=1))
assert fb == ob, pqwalk.first_difference(fb, ob)
print("split ok", len(fb))
"""


def test_writer_batches_split_at_job_size():
    """Bulk batches larger than the room left in the fill buffer (gap + job size + 64 MiB) are
    split where they stop fitting (writer.cpp write_bulk_split) instead of growing the buffer.
    With 2 MiB jobs the buffers hold ~130 MiB, so each ~74 MB batch is split; row groups cross
    the job boundaries and the file must not change.  Runs in a child process: the job size is
    read once per process (KPW_STAGE_FLUSH_MB)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    paths = ":".join(os.path.join(root, d) for d in ("synth", "oracle", "tests", "kafka-parquet-writer_amd", ""))
    env = dict(os.environ, KPW_STAGE_FLUSH_MB="2")
    r = subprocess.run([sys.executable, "-c", _SPLIT_CHILD, paths], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "split ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


_EAGER_CHILD = r"""
import sys
sys.path[:0] = sys.argv[1].split(":")
import kpw, oracle, pqwalk, synth
schema = synth.REC8
n = 1_500_000
data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE0B, n)
for block in (1 << 20, 8 << 20):
    props = kpw.ParquetProperties(block_size=block, compression_codec_name=1)
    pf = kpw.ParquetFile(None, kpw.Schema(schema.message_name, schema.columns, schema.proto_class), props)
    for i in range(0, n, 100_000):
        j = min(n, i + 100_000)
        pf.write_batch((data[int(offs[i]):int(offs[j])], offs[i:j + 1] - offs[i]))
    pf.close()
    fb = pf.file_bytes()
    ob = oracle.encode_file(schema, data, offs, oracle.make_props(block_size=block, codec=1))
    assert fb == ob, pqwalk.first_difference(fb, ob)
print("eager ok")
"""


def test_writer_eager_jobs():
    """Eager jobs (writer.cpp eager_job_bytes): a fill buffer past KPW_EAGER_MB is submitted as
    soon as an encode worker idles, so job boundaries depend on timing.  With 1 MiB eager jobs
    and 6 MB batches nearly every batch becomes a job whose open row group is carried into the
    next; the file must stay byte-identical to the oracle's at either row-group size.  Runs in a
    child process (the job size is read once per process)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    paths = ":".join(os.path.join(root, d) for d in ("synth", "oracle", "tests", "kafka-parquet-writer_amd", ""))
    env = dict(os.environ, KPW_EAGER_MB="1", KPW_STAGE_FLUSH_MB="64")
    r = subprocess.run([sys.executable, "-c", _EAGER_CHILD, paths], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "eager ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


_LEN_CHILD = r"""
import sys
import numpy as np
sys.path[:0] = sys.argv[1].split(":")
import kpw, oracle, pqwalk, synth

def varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)

def rec(i, qlen):
    q = bytes((65 + (i + k) % 26) for k in range(qlen))
    return b"\x0a" + varint(len(q)) + q + b"\x10" + varint(1700000000000 + i)

schema = synth.SAMPLE
for name, big in (("u8", 0), ("u16", 300), ("u32", 70000)):
    recs = [rec(i, big if big and i % 97 == 5 else 3 + i % 40) for i in range(3000)]
    offs = np.zeros(len(recs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(r) for r in recs])
    data = np.frombuffer(b"".join(recs), dtype=np.uint8)
    props = kpw.ParquetProperties(block_size=64 << 10, compression_codec_name=1)
    pf = kpw.ParquetFile(None, kpw.Schema(schema.message_name, schema.columns, schema.proto_class), props)
    for i in range(0, len(recs), 500):
        j = min(len(recs), i + 500)
        pf.write_batch((data[int(offs[i]):int(offs[j])], offs[i:j + 1] - offs[i]))
    pf.close()
    fb = pf.file_bytes()
    ob = oracle.encode_file(schema, data, offs, oracle.make_props(block_size=64 << 10, codec=1))
    assert fb == ob, name + ": " + str(pqwalk.first_difference(fb, ob))
print("lengths ok")
"""


def test_writer_record_length_widths():
    """Record offsets cross PCIe as u8 / u16 / u32 lengths (writer.cpp upload_offsets): a job
    whose records all fit a byte goes as u8, a 300-byte or 70 KB record sends the job through
    u16 / u32.  Bulk writes of 500 records (KPW_MODEL_MAX_BATCH=8, so they skip the per-record
    model) with such records every 97th; each file byte-identical to the oracle's."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    paths = ":".join(os.path.join(root, d) for d in ("synth", "oracle", "tests", "kafka-parquet-writer_amd", ""))
    env = dict(os.environ, KPW_MODEL_MAX_BATCH="8", KPW_STAGE_FLUSH_MB="1", KPW_EAGER_MB="-1")
    r = subprocess.run([sys.executable, "-c", _LEN_CHILD, paths], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "lengths ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


@pytest.mark.parametrize("pattern", ["random", "zeros", "period3", "text", "mixed"])
def test_gzip_patterns(pattern):
    """K7 GZIP on byte patterns that exercise zlib's corner cases: stored blocks (incompressible),
    maximal matches and long chains (zeros, short periods), lazy matches and dynamic trees (text),
    window slides and blocks of 16383 symbols (every page here is > 64 KiB)."""
    rng = np.random.default_rng(7)
    n = 60000
    if pattern == "random":
        vals = [rng.integers(0, 256, 40, dtype=np.uint8).tobytes() for _ in range(n)]
    elif pattern == "zeros":
        vals = [bytes(24) for _ in range(n)]
    elif pattern == "period3":
        vals = [b"abc" * 11 for _ in range(n)]
    elif pattern == "text":
        words = [b"kafka", b"parquet", b"writer", b"gzip", b"deflate", b"page", b"row", b"group"]
        vals = [b" ".join(words[int(k)] for k in rng.integers(0, 8, 6)) for _ in range(n)]
    else:
        vals = [rng.integers(0, 256, 40, dtype=np.uint8).tobytes() if i % 3 == 0 else b"x" * (i % 50) for i in range(n)]
    # one required bytes field (1) carries the pattern bytes
    recs = [b"\x0a" + protoutil_varint(len(v)) + v for v in vals]
    from types import SimpleNamespace
    s = SimpleNamespace(message_name="test.Bytes", columns=[("payload", 1, synth.BYTES, synth.REQUIRED)],
                        proto_class="test.Bytes")
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum([len(r) for r in recs], out=offs[1:])
    data = np.frombuffer(b"".join(recs), dtype=np.uint8)
    errs = gh.compare_pages(s, data, offs, codec=2, dictionary=False)
    assert not errs, "\n".join(errs[:12])


def protoutil_varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)
