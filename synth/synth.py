"""Synthetic Kafka record values + schema catalogue (test/bench infrastructure).

Schemas mirror SURVEY.md §8d.  A schema is a list of
(name, field_number, proto_type, label) tuples in proto declaration order plus a
message name, exactly what a host fills from the proto Descriptor
(ProtoSchemaConverter, parquet-mr 1.10.1; reference ParquetFile.java:96-99).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libkpw_synth.so")

# descriptor.proto Type / Label numbering (include/kpw_types.h)
DOUBLE, FLOAT, INT64, UINT64, INT32, FIXED64, FIXED32, BOOL, STRING = 1, 2, 3, 4, 5, 6, 7, 8, 9
BYTES, UINT32, SFIXED32, SFIXED64, SINT32, SINT64 = 12, 13, 15, 16, 17, 18
OPTIONAL, REQUIRED = 1, 2

KIND_SAMPLE, KIND_REC8, KIND_HIGHCARD, KIND_WIDE = 0, 1, 2, 3


class Schema:
    def __init__(self, message_name, columns, proto_class=None):
        self.message_name = message_name
        self.columns = list(columns)
        self.proto_class = proto_class or message_name


# src/test/resources/test-message.proto:5-10
SAMPLE = Schema("SampleMessage", [
    ("query", 1, STRING, REQUIRED),
    ("timestamp", 2, INT64, REQUIRED),
    ("page_number", 3, INT32, OPTIONAL),
    ("result_per_page", 4, INT32, OPTIONAL),
], proto_class="ir.sahab.kafka.test.proto.TestMessage$SampleMessage")

REC8 = Schema("kpw.bench.Rec8", [
    ("ts", 1, INT64, REQUIRED),
    ("user_id", 2, INT32, REQUIRED),
    ("status", 3, INT32, OPTIONAL),
    ("price", 4, DOUBLE, REQUIRED),
    ("score", 5, DOUBLE, OPTIONAL),
    ("key16", 6, STRING, REQUIRED),
    ("region", 7, STRING, OPTIONAL),
    ("flag", 8, BOOL, OPTIONAL),
], proto_class="kpw.bench.Rec8Proto$Rec8")

HIGHCARD = Schema("kpw.bench.HighCard", [
    ("ts", 1, INT64, REQUIRED),
    ("uuid", 2, STRING, REQUIRED),
    ("blob", 3, STRING, REQUIRED),
    ("code", 4, INT32, OPTIONAL),
], proto_class="kpw.bench.HighCardProto$HighCard")


def _wide_columns():
    cols = [("ts", 1, INT64, REQUIRED)]
    for f in range(2, 201):
        if f <= 81:
            cols.append(("c%03d" % f, f, INT64, OPTIONAL))
        elif f <= 141:
            cols.append(("d%03d" % f, f, DOUBLE, OPTIONAL))
        else:
            cols.append(("s%03d" % f, f, STRING, OPTIONAL))
    return cols


WIDE = Schema("kpw.bench.Wide", _wide_columns(), proto_class="kpw.bench.WideProto$Wide")

SCHEMAS = {KIND_SAMPLE: SAMPLE, KIND_REC8: REC8, KIND_HIGHCARD: HIGHCARD, KIND_WIDE: WIDE}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("synth library missing: run `make -C synth`")
        L = ctypes.CDLL(LIB_PATH)
        for fn in (L.synth_sizes, L.synth_fill):
            fn.restype = ctypes.c_int
        _lib = L
    return _lib


def generate(kind, seed, n, start=0, param=0, alloc=None):
    """Return (data: np.uint8[], offsets: np.uint64[n+1]) for records start..start+n-1.
    alloc(nbytes) -> uint8 array to generate into (e.g. kpw.pinned_empty); default numpy."""
    L = lib()
    sizes = np.empty(n, dtype=np.uint32)
    L.synth_sizes(ctypes.c_int(kind), ctypes.c_uint64(seed), ctypes.c_uint64(start), ctypes.c_uint64(n),
                  ctypes.c_int(param), sizes.ctypes.data_as(ctypes.c_void_p))
    offsets = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(sizes, out=offsets[1:])
    del sizes
    data = alloc(int(offsets[-1])) if alloc else np.empty(int(offsets[-1]), dtype=np.uint8)
    L.synth_fill(ctypes.c_int(kind), ctypes.c_uint64(seed), ctypes.c_uint64(start), ctypes.c_uint64(n),
                 ctypes.c_int(param), offsets.ctypes.data_as(ctypes.c_void_p), data.ctypes.data_as(ctypes.c_void_p))
    return data, offsets


def per_record_loop(kind, write_fn, data_size_fn, handle, data, offsets, start, n, max_file_size):
    """The reference WorkerThread loop in C (synth/loop.c): records [start, start+n) written
    ONE at a time, getDataSize() after each, stop after the first with getDataSize() >=
    max_file_size.  kind "kpw": write_fn / data_size_fn are kpw_writer_write /
    kpw_writer_data_size (ctypes functions); "oracle": kpwo_write / kpwo_data_size.
    Returns (records written, full, status, last getDataSize())."""
    L = lib()
    fn = L.loop_kpw if kind == "kpw" else L.loop_oracle
    fn.restype = ctypes.c_uint64
    fn.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64,
                                            ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                            ctypes.POINTER(ctypes.c_int64)]
    full, st, last = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int64(0)
    got = fn(ctypes.cast(write_fn, ctypes.c_void_p), ctypes.cast(data_size_fn, ctypes.c_void_p), handle,
             data.ctypes.data, offsets.ctypes.data + 8 * start, n, max_file_size, ctypes.byref(full), ctypes.byref(st),
             ctypes.byref(last))
    return int(got), bool(full.value), st.value, last.value


def records(data, offsets):
    return [bytes(data[int(offsets[i]):int(offsets[i + 1])]) for i in range(len(offsets) - 1)]


def pack(recs):
    """list[bytes] -> (data, offsets)"""
    offsets = np.zeros(len(recs) + 1, dtype=np.uint64)
    if recs:
        np.cumsum([len(r) for r in recs], out=offsets[1:])
    data = np.frombuffer(b"".join(recs), dtype=np.uint8).copy() if recs else np.zeros(0, np.uint8)
    return data, offsets
