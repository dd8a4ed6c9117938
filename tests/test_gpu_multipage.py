"""GPU parity in the multi-page regime (PARQUET_1_0, pageSize < blockSize): pages cut inside a
row group by ColumnWriterV1.accountForValueWritten, the dictionary kept across a chunk's pages
with a per-page bit width, fallback to PLAIN from the page where the dictionary crosses
dictPageSize, isCompressionSatisfying on the first page only, and row groups cut by a size
check that counts flushed pages by their header + compressed bytes.  Every page byte-identical
to the CPU oracle (oracle/oracle_core.c colw_account / check_block_size)."""
import io
import os

import pyarrow.parquet as pq
import pytest

import gpu_helpers as gh
import oracle
import protoutil
import synth

pytestmark = pytest.mark.gpu
KiB = 1024
MiB = 1024 * 1024

CASES = [
    ("sample", synth.KIND_SAMPLE, 0, 6000),
    ("sample_nulls", synth.KIND_SAMPLE, 30, 6000),
    ("rec8", synth.KIND_REC8, 0, 40000),
    ("highcard", synth.KIND_HIGHCARD, 0, 6000),
    ("wide", synth.KIND_WIDE, 0, 1500),
]


@pytest.mark.parametrize("name,kind,param,n", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("codec", [0, 1], ids=["uncompressed", "snappy"])
@pytest.mark.parametrize("block_size,page_size", [(256 * KiB, 8 * KiB), (128 * MiB, 16 * KiB), (64 * KiB, 1024)],
                         ids=["rg256K_p8K", "rg128M_p16K", "rg64K_p1K"])
def test_multipage_matches_oracle(name, kind, param, n, codec, block_size, page_size):
    schema = synth.SCHEMAS[kind]
    data, offs = synth.generate(kind, 0xC0FFEE41 + kind, n, param=param)
    errs = gh.compare_pages(schema, data, offs, codec=codec, block_size=block_size, page_size=page_size)
    assert not errs, "\n".join(errs[:12])


def _pairs_records(n):
    # every query value twice in a row: the first page's dictionary is worth keeping
    # (isCompressionSatisfying), and the dictionary crosses 1 MiB after ~31k distinct
    # 30-byte values, many 64 KiB pages into the chunk
    cls = protoutil.message_class(synth.SAMPLE)
    recs = [cls(query="query-%024d" % (i // 2), timestamp=1700000000000 + i,
                page_number=i % 7).SerializeToString() for i in range(n)]
    return synth.pack(recs)


def test_multipage_fallback_mid_chunk():
    # earlier pages keep PLAIN_DICTIONARY ids (bit width growing page by page), the page where
    # the dictionary crosses dictPageSize and every later one is PLAIN, and the dictionary page
    # holds the entries of the last dictionary-encoded page
    import pqwalk
    data, offs = _pairs_records(80000)
    for codec in (0, 1):
        errs = gh.compare_pages(synth.SAMPLE, data, offs, codec=codec, page_size=64 * KiB)
        assert not errs, "\n".join(errs[:12])
    fb = oracle.encode_file(synth.SAMPLE, data, offs, oracle.make_props(codec=1, page_size=64 * KiB))
    encs = [p["header"][5][2] for p in pqwalk.pages(fb) if p["col"] == 0 and p["header"][1] == 0]
    assert encs[0] == 2 and encs[-1] == 0, encs   # PLAIN_DICTIONARY first, PLAIN after the fallback


# (codec, row-group size, dictPageSize in KiB): for _pairs_records(60000) and 16 KiB pages the
# oracle's query column crosses dictPageSize in every row group's first page (4), a middle page
# (24, 70, 160, 240, 256), the last page (258, 404), just after the row-group end (inside the
# speculative pass's range: 262, 408), or never within a row group (400, 412)
SPLICE_CASES = [(0, 160, 4), (0, 160, 24), (0, 160, 160), (0, 160, 240), (0, 160, 256), (0, 160, 258), (0, 160, 262),
                (0, 160, 400), (1, 160, 4), (1, 160, 70), (1, 160, 404), (1, 160, 408), (1, 160, 412), (2, 64, 4),
                (2, 64, 100), (2, 64, 150), (2, 64, 200)]


@pytest.mark.parametrize("codec,rg_kib,dict_kib", SPLICE_CASES, ids=["c%d_rg%dK_d%dK" % c for c in SPLICE_CASES])
def test_multipage_splice_dictionary_crossing(codec, rg_kib, dict_kib):
    # many row groups cut inside one batch, so every exact pass but the last is a splice
    # (engine_mp.cpp: only each column's last page and its dictionary page re-encoded): the
    # dictionary crosses dictPageSize in the first page (every page PLAIN), in a middle page,
    # in the last page of the row group, after its end (the last page keeps its ids), or never
    data, offs = _pairs_records(60000)
    kw = dict(codec=codec, block_size=rg_kib * KiB, page_size=16 * KiB, dict_page_size=dict_kib * KiB)
    fb = oracle.encode_file(synth.SAMPLE, data, offs, gh.oracle_props(**kw))
    assert len(gh.oracle_row_groups(fb)) >= 3
    errs = gh.compare_to_file(synth.SAMPLE, data, offs, fb, **kw)[0]
    assert not errs, "\n".join(errs[:12])


@pytest.mark.parametrize("name,kind,param,n", CASES, ids=[c[0] for c in CASES])
def test_multipage_splice_gzip(name, kind, param, n):
    # the splice with GZIP members (kept pages copied, the last page and dictionary page deflated)
    schema = synth.SCHEMAS[kind]
    data, offs = synth.generate(kind, 0xC0FFEE44 + kind, n, param=param)
    errs = gh.compare_pages(schema, data, offs, codec=2, block_size=128 * KiB, page_size=4 * KiB)
    assert not errs, "\n".join(errs[:12])


@pytest.mark.parametrize("mode", ["file", "data_size"])
def test_multipage_lazy_open_jobs(mode):
    # write-path jobs of ~6 MB (KPW_EAGER_MB=4, in a child process: the knob is read once) stop
    # after their last row-group cut and carry the rest to the next job without planning it
    # (Engine::lazy_open); getDataSize after a batch then plans the open row group on demand
    import subprocess
    import sys
    env = dict(os.environ, KPW_EAGER_MB="4")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "lazy_open_child.py"), mode, "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "LAZY_OPEN_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


@pytest.mark.parametrize("page_size", [64, 300])
def test_multipage_tiny_pages(page_size):
    # pages of a handful of values: every size check cuts, next check = valueCount / 2
    data, offs = synth.generate(synth.KIND_SAMPLE, 3, 3000, param=30)
    errs = gh.compare_pages(synth.SAMPLE, data, offs, codec=1, block_size=32 * KiB, page_size=page_size)
    assert not errs, "\n".join(errs[:12])


def test_multipage_rowgroups_by_compressed_pages():
    # 1 MiB pages in 4 MiB row groups: after the first page cuts the row-group check counts
    # Snappy-compressed pages, so row groups hold more records than raw bytes suggest
    schema = synth.REC8
    data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE42, 300000)
    errs = gh.compare_pages(schema, data, offs, codec=1, block_size=4 * MiB, page_size=1 * MiB)
    assert not errs, "\n".join(errs[:12])


def test_multipage_writer_file_identical():
    import kpw
    import pqwalk
    schema = synth.REC8
    data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE43, 30000, param=0)
    props = kpw.ParquetProperties(block_size=256 * 1024, page_size=16 * 1024, compression_codec_name=1)
    fb = gh.gpu_file(schema, data, offs, props, batches=3)
    ob = oracle.encode_file(schema, data, offs, oracle.make_props(block_size=256 * 1024, page_size=16 * 1024, codec=1))
    assert fb == ob, pqwalk.first_difference(fb, ob)
    tbl = pq.read_table(io.BytesIO(fb))
    assert protoutil.table_columns(tbl, schema) == protoutil.decode_columns(schema, synth.records(data, offs))


# ------------------------------------------------------------------ PARQUET_2_0 (A10 / f4)
# ColumnWriteStoreV2.sizeCheck cuts pages for the whole store (a column within 10% of pageSize
# writes its page; next check at rowCount + min(max(min rowsToFillPage / 2, 100), 10000)),
# pages are DataPageV2 (width-0 repetition levels on every page, REQUIRED columns' width-0
# definition levels, RLE booleans counted by their RLE bytes), DELTA fallback streams restart
# on every page, and the row-group check counts flushed pages by header + levels + compressed
# values.  Unreachable from the reference (ParquetFile.java:42-50 never selects v2): parity
# against the oracle's restatement.

@pytest.mark.parametrize("name,kind,param,n", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("codec", [0, 1], ids=["uncompressed", "snappy"])
@pytest.mark.parametrize("block_size,page_size", [(256 * KiB, 8 * KiB), (128 * MiB, 16 * KiB), (64 * KiB, 1024)],
                         ids=["rg256K_p8K", "rg128M_p16K", "rg64K_p1K"])
def test_v2_multipage_matches_oracle(name, kind, param, n, codec, block_size, page_size):
    schema = synth.SCHEMAS[kind]
    data, offs = synth.generate(kind, 0xC0FFEE51 + kind, n, param=param)
    errs = gh.compare_pages(schema, data, offs, codec=codec, block_size=block_size, page_size=page_size, writer_version=2)
    assert not errs, "\n".join(errs[:12])


def test_v2_multipage_fallback_mid_chunk():
    # the page where the dictionary crosses dictPageSize and every later page fall back to
    # DELTA_BYTE_ARRAY (query) with a fresh stream per page
    import pqwalk
    data, offs = _pairs_records(80000)
    for codec in (0, 1):
        errs = gh.compare_pages(synth.SAMPLE, data, offs, codec=codec, page_size=64 * KiB, writer_version=2)
        assert not errs, "\n".join(errs[:12])
    fb = oracle.encode_file(synth.SAMPLE, data, offs, oracle.make_props(codec=1, page_size=64 * KiB, writer_version=2))
    encs = [p["header"][8][4] for p in pqwalk.pages(fb) if p["col"] == 0 and p["header"][1] == 3]
    assert encs[0] == 8 and encs[-1] == 7, encs   # RLE_DICTIONARY first, DELTA_BYTE_ARRAY after the fallback


def test_v2_multipage_writer_file_identical():
    import kpw
    import pqwalk
    schema = synth.REC8
    data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE53, 30000, param=0)
    props = kpw.ParquetProperties(block_size=256 * 1024, page_size=16 * 1024, compression_codec_name=1, writer_version=2)
    fb = gh.gpu_file(schema, data, offs, props, batches=3)
    ob = oracle.encode_file(schema, data, offs, oracle.make_props(block_size=256 * 1024, page_size=16 * 1024, codec=1,
                                                                  writer_version=2))
    assert fb == ob, pqwalk.first_difference(fb, ob)
    tbl = pq.read_table(io.BytesIO(fb))
    assert protoutil.table_columns(tbl, schema) == protoutil.decode_columns(schema, synth.records(data, offs))
