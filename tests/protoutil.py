"""Independent proto2 decoding for tests, via google.protobuf dynamic messages.

This is the Python-side stand-in for the reference test's ProtoParquetReader/protobuf
equality (ParquetTestUtils.java:28-47, KafkaProtoParquetWriterTest.java:136-139): the
expected column values come from protobuf's own parser, not from the oracle's decoder.
"""
import struct

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_cache = {}


def message_class(schema):
    key = (schema.message_name, tuple(schema.columns))
    if key in _cache:
        return _cache[key]
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = "kpw_test_%d.proto" % len(_cache)
    fdp.syntax = "proto2"
    parts = schema.message_name.split(".")
    if len(parts) > 1:
        fdp.package = ".".join(parts[:-1])
    msg = fdp.message_type.add()
    msg.name = parts[-1]
    for name, fno, pt, label in schema.columns:
        f = msg.field.add()
        f.name = name
        f.number = fno
        f.type = pt
        f.label = label
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    desc = pool.FindMessageTypeByName(schema.message_name)
    cls = message_factory.GetMessageClass(desc)
    _cache[key] = cls
    return cls


def _canon_double(x):
    # parquet-mr writes Double.doubleToLongBits: NaN canonicalised
    if x != x:
        return struct.unpack("<d", struct.pack("<Q", 0x7FF8000000000000))[0]
    return x


def decode_columns(schema, recs):
    """Return {column_name: list of python values or None} as the Parquet file must hold them."""
    cls = message_class(schema)
    cols = {c[0]: [] for c in schema.columns}
    for r in recs:
        m = cls()
        m.ParseFromString(r)
        for name, fno, pt, label in schema.columns:
            if label == 1 and not m.HasField(name):
                cols[name].append(None)
                continue
            v = getattr(m, name)
            if pt in (2, 1):
                v = _canon_double(v)
            if pt == 4:   # uint64 stored as INT64 bits -> signed view
                v = v - (1 << 64) if v >= (1 << 63) else v
            if pt == 13:  # uint32 stored as INT32 bits -> signed view
                v = v - (1 << 32) if v >= (1 << 31) else v
            if pt == 9:
                v = v.encode("utf-8") if isinstance(v, str) else v
            cols[name].append(v)
    return cols


def table_columns(table, schema):
    """pyarrow Table -> {name: list} with strings as bytes (to compare bytes exactly)."""
    out = {}
    for name, fno, pt, label in schema.columns:
        col = table.column(name)
        vals = col.to_pylist()
        if pt == 9:
            vals = [v.encode("utf-8") if isinstance(v, str) else v for v in vals]
        out[name] = vals
    return out
