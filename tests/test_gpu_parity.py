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
@pytest.mark.parametrize("codec", [0, 1], ids=["uncompressed", "snappy"])
@pytest.mark.parametrize("block_size", [128 * MiB, 64 * 1024], ids=["rg128M", "rg64K"])
def test_pages_match_oracle(name, kind, param, n, codec, block_size):
    schema = synth.SCHEMAS[kind]
    data, offs = synth.generate(kind, 0xC0FFEE01 + kind, n, param=param)
    errs = gh.compare_pages(schema, data, offs, codec=codec, block_size=block_size)
    assert not errs, "\n".join(errs[:12])


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


@pytest.mark.parametrize("n", [1, 7, 8, 9, 63, 64, 65, 100, 101, 255])
def test_tiny_batches(n):
    data, offs = synth.generate(synth.KIND_REC8, 99, n)
    errs = gh.compare_pages(synth.REC8, data, offs, codec=1, block_size=4096)
    assert not errs, "\n".join(errs[:12])


@pytest.mark.parametrize("kind", [synth.KIND_SAMPLE, synth.KIND_REC8])
@pytest.mark.parametrize("codec", [0, 1])
def test_writer_file_identical(kind, codec):
    """The ParquetFile drop-in writes the same file bytes as the oracle, across several
    write batches (open row groups carried between encoder batches)."""
    schema = synth.SCHEMAS[kind]
    data, offs = synth.generate(kind, 0xC0FFEE01, 20000)
    import kpw
    props = kpw.ParquetProperties(block_size=256 * 1024, compression_codec_name=codec)
    fb = gh.gpu_file(schema, data, offs, props, batches=3)
    ob = oracle.encode_file(schema, data, offs, oracle.make_props(block_size=256 * 1024, codec=codec))
    import pqwalk
    assert fb == ob, pqwalk.first_difference(fb, ob)
    tbl = pq.read_table(io.BytesIO(fb))
    assert protoutil.table_columns(tbl, schema) == protoutil.decode_columns(schema, synth.records(data, offs))


def test_invalid_record_cuts_batch():
    import kpw
    good = synth.records(*synth.generate(synth.KIND_SAMPLE, 1, 50))
    bad = b"\x10\x01"  # missing required query
    pf = kpw.ParquetFile(None, kpw.Schema(synth.SAMPLE.message_name, synth.SAMPLE.columns))
    pf.write_batch(good + [bad] + good[:5])
    with pytest.raises(kpw.InvalidProtoError) as e:
        pf.get_data_size()
    assert e.value.record == 50
    pf.close()
    tbl = pq.read_table(io.BytesIO(pf.file_bytes()))
    assert tbl.num_rows == 50
