"""K1 (k_decode) against the reference's parse semantics, through the C-ABI.

The record lists are the ones the oracle is pinned with (tests/wire_cases.py, shared with
test_oracle.py): protobuf-java's generated parse loop (TestMessage.java:85-139) and
isInitialized (:263-278) as reached from KafkaProtoParquetWriter.java:268-276.  Accepted
records must give pages byte-identical to the oracle; rejected ones must stop the batch at
the same record index as the oracle's write loop, with the records before it encoded
identically (encoder path) and written identically (ParquetFile path).
"""
import io

import numpy as np
import pyarrow.parquet as pq
import pytest

import gpu_helpers as gh
import oracle
import pqwalk
import synth
import wire_cases

pytestmark = pytest.mark.gpu
MiB = 1024 * 1024


def _goods(n, seed=1):
    return synth.records(*synth.generate(synth.KIND_SAMPLE, seed, n, param=30))


@pytest.mark.parametrize("codec", [0, 1], ids=["uncompressed", "snappy"])
def test_accepted_edge_cases_pages(codec):
    recs = [r for _, r in wire_cases.accepted()]
    data, offs = synth.pack(recs)
    errs = gh.compare_pages(synth.SAMPLE, data, offs, codec=codec)
    assert not errs, "\n".join(errs[:12])


@pytest.mark.parametrize("block_size", [128 * MiB, 16 * 1024], ids=["rg128M", "rg16K"])
def test_accepted_edge_cases_many_waves(block_size):
    """Every accepted case at every lane position of several waves and blocks (records
    interleaved with canonical ones, 5000 records)."""
    cases = [r for _, r in wire_cases.accepted()]
    goods = _goods(5000, seed=7)
    rng = np.random.default_rng(11)
    recs = [cases[int(rng.integers(0, len(cases)))] if rng.random() < 0.4 else g for g in goods]
    data, offs = synth.pack(recs)
    errs = gh.compare_pages(synth.SAMPLE, data, offs, codec=1, block_size=block_size)
    assert not errs, "\n".join(errs[:12])


def test_accepted_edge_cases_file_identical():
    import kpw
    recs = [r for _, r in wire_cases.accepted()] * 50
    data, offs = synth.pack(recs)
    props = kpw.ParquetProperties(block_size=8 * 1024, compression_codec_name=1)
    fb = gh.gpu_file(synth.SAMPLE, data, offs, props, batches=3)
    ob = oracle.encode_file(synth.SAMPLE, data, offs, oracle.make_props(block_size=8 * 1024, codec=1))
    assert fb == ob, pqwalk.first_difference(fb, ob)


INVALID = wire_cases.invalid()


@pytest.mark.parametrize("pos", [0, 1, 63, 64, 255, 256, 700])
@pytest.mark.parametrize("label,bad", INVALID, ids=[c[0] for c in INVALID])
def test_invalid_record_index_and_prefix(label, bad, pos):
    """Encoder path: invalid_record == the oracle's stop index; the pages of every record
    before it byte-identical to the oracle's file of that prefix."""
    goods = _goods(pos + 40, seed=3)
    recs = goods[:pos] + [bad] + goods[pos:]
    data, offs = synth.pack(recs)
    w = oracle.OracleWriter(synth.SAMPLE, gh.oracle_props(codec=1, block_size=4096))
    st, nw = w.write_batch(data, offs)
    assert st == -3 and nw == pos
    w.close()
    fb = w.file_bytes()
    errs, info = gh.compare_to_file(synth.SAMPLE, data, offs, fb, codec=1, block_size=4096)
    assert info.invalid_record == pos
    assert not errs, "\n".join(errs[:12])


@pytest.mark.parametrize("label,bad", INVALID, ids=[c[0] for c in INVALID])
def test_invalid_record_parquet_file(label, bad):
    """ParquetFile path: the error surfaces as InvalidProtoError with the record index, and
    the closed file holds exactly the records before it (the oracle's file)."""
    import kpw
    goods = _goods(300, seed=5)
    pos = 137
    pf = kpw.ParquetFile(None, kpw.Schema(synth.SAMPLE.message_name, synth.SAMPLE.columns, synth.SAMPLE.proto_class),
                         kpw.ParquetProperties(block_size=4096, compression_codec_name=1))
    with pytest.raises(kpw.InvalidProtoError) as e:   # small write: raised by the write itself
        pf.write_batch(goods[:pos] + [bad] + goods[pos:])
    assert e.value.record == pos
    assert pf.get_num_written_records() == pos
    pf.close()
    got = pf.file_bytes()
    data, offs = synth.pack(goods[:pos])
    want = oracle.encode_file(synth.SAMPLE, data, offs, oracle.make_props(block_size=4096, codec=1))
    assert got == want, pqwalk.first_difference(got, want)
    assert pq.read_table(io.BytesIO(got)).num_rows == pos


def test_footer_descriptor_matches_reference():
    """The GPU writer's footer carries the reference's own descriptor (TestMessage.java:750-755,
    tests/golden/test_message_descriptor.json) as parquet.proto.descriptor."""
    import json
    import os
    import kpw
    desc = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                       "test_message_descriptor.json")))
    data, offs = synth.generate(synth.KIND_SAMPLE, 3, 200)
    fb = gh.gpu_file(synth.SAMPLE, data, offs, kpw.ParquetProperties())
    kv = {e[1].decode(): e[2].decode() for e in pqwalk.footer(fb)[5]}
    assert kv["parquet.proto.descriptor"] == desc["descriptor_text"]
    assert kv["parquet.proto.class"] == desc["proto_class"]
    assert pqwalk.footer(fb)[2][0][4].decode() == desc["message_full_name"]


def test_c1_one_million_records_uncompressed():
    """C1: 1 M Rec8 records, seed 0xC0FFEE01, UNCOMPRESSED, dictionary on,
    128 MiB row groups and pages — pages and the whole file byte-identical to the oracle."""
    import kpw
    data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE01, 1_000_000)
    errs = gh.compare_pages(synth.REC8, data, offs, codec=0)
    assert not errs, "\n".join(errs[:12])
    props = kpw.ParquetProperties(compression_codec_name=0)
    fb = gh.gpu_file(synth.REC8, data, offs, props, batches=4)
    ob = oracle.encode_file(synth.REC8, data, offs, oracle.make_props(codec=0))
    assert fb == ob, pqwalk.first_difference(fb, ob)


@pytest.mark.parametrize("label,bad", INVALID[:3] + INVALID[-2:], ids=[c[0] for c in INVALID[:3] + INVALID[-2:]])
def test_invalid_record_bulk_write(label, bad):
    """Bulk path (a write of > 65536 records, validated on the GPU): the error surfaces at the
    next call with the record index, and the file holds exactly the records before it."""
    import kpw
    goods = _goods(100000, seed=9)
    pos = 70001
    pf = kpw.ParquetFile(None, kpw.Schema(synth.SAMPLE.message_name, synth.SAMPLE.columns, synth.SAMPLE.proto_class),
                         kpw.ParquetProperties(block_size=256 * 1024, compression_codec_name=1))
    pf.write_batch(goods[:pos] + [bad] + goods[pos:])
    with pytest.raises(kpw.InvalidProtoError) as e:
        pf.get_data_size()
    assert e.value.record == pos
    assert pf.get_num_written_records() == pos
    pf.close()
    data, offs = synth.pack(goods[:pos])
    want = oracle.encode_file(synth.SAMPLE, data, offs, oracle.make_props(block_size=256 * 1024, codec=1))
    got = pf.file_bytes()
    assert got == want, pqwalk.first_difference(got, want)
