"""ctypes wrapper of the CPU ORACLE (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / CPU baseline.  See kpw_oracle.h for what it restates
and how it is pinned.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libkpw_oracle.so")


class ColumnDesc(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("field_number", ctypes.c_int32),
                ("proto_type", ctypes.c_int32), ("label", ctypes.c_int32)]


class SchemaC(ctypes.Structure):
    _fields_ = [("message_name", ctypes.c_char_p), ("proto_class", ctypes.c_char_p),
                ("num_columns", ctypes.c_int32), ("columns", ctypes.POINTER(ColumnDesc))]


class PropsC(ctypes.Structure):
    _fields_ = [("block_size", ctypes.c_int64), ("page_size", ctypes.c_int32),
                ("dictionary_page_size", ctypes.c_int32), ("enable_dictionary", ctypes.c_int32),
                ("codec", ctypes.c_int32), ("writer_version", ctypes.c_int32), ("reserved0", ctypes.c_int32),
                ("dfs_block_size", ctypes.c_int64), ("max_padding_size", ctypes.c_int64)]


UNCOMPRESSED, SNAPPY, GZIP = 0, 1, 2
MiB = 1024 * 1024


def make_props(block_size=128 * MiB, page_size=128 * MiB, codec=UNCOMPRESSED, enable_dictionary=True,
               dictionary_page_size=1 * MiB, dfs_block_size=0, max_padding_size=8 * MiB, writer_version=1):
    return PropsC(block_size, page_size, dictionary_page_size, 1 if enable_dictionary else 0, codec, writer_version, 0,
                  dfs_block_size, max_padding_size)


def make_schema(schema):
    """schema: synth.Schema-like (message_name, columns, proto_class). Returns (struct, keepalive)."""
    cols = (ColumnDesc * len(schema.columns))()
    keep = []
    for i, (name, fno, pt, label) in enumerate(schema.columns):
        b = name.encode()
        keep.append(b)
        cols[i] = ColumnDesc(b, fno, pt, label)
    mn = schema.message_name.encode()
    pc = (schema.proto_class or schema.message_name).encode()
    keep += [mn, pc, cols]
    return SchemaC(mn, pc, len(schema.columns), cols), keep


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle library missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        L.kpwo_open.restype = ctypes.c_void_p
        L.kpwo_open.argtypes = [ctypes.POINTER(SchemaC), ctypes.POINTER(PropsC), ctypes.POINTER(ctypes.c_int)]
        L.kpwo_write.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.kpwo_write_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.POINTER(ctypes.c_uint64)]
        L.kpwo_write_until_full.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                            ctypes.c_int64, ctypes.POINTER(ctypes.c_uint64),
                                            ctypes.POINTER(ctypes.c_int)]
        L.kpwo_data_size.restype = ctypes.c_int64
        L.kpwo_data_size.argtypes = [ctypes.c_void_p]
        L.kpwo_num_records.restype = ctypes.c_int64
        L.kpwo_num_records.argtypes = [ctypes.c_void_p]
        L.kpwo_close.argtypes = [ctypes.c_void_p]
        L.kpwo_file_bytes.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                      ctypes.POINTER(ctypes.c_uint64)]
        L.kpwo_num_row_groups.argtypes = [ctypes.c_void_p]
        L.kpwo_free.argtypes = [ctypes.c_void_p]
        L.kpwo_rle_encode.restype = ctypes.c_int64
        L.kpwo_rle_encode.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_uint64]
        L.kpwo_delta_encode.restype = ctypes.c_int64
        L.kpwo_delta_encode.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_uint64]
        L.kpwo_snappy_compress.restype = ctypes.c_int64
        L.kpwo_snappy_compress.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
        for fn in (L.kpwo_gzip_compress, L.kpwo_deflate_raw):
            fn.restype = ctypes.c_int64
            fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
        L.kpwo_gzip_bound.restype = ctypes.c_uint64
        L.kpwo_gzip_bound.argtypes = [ctypes.c_uint64]
        L.kpwo_snappy_max_compressed_length.restype = ctypes.c_uint64
        L.kpwo_snappy_max_compressed_length.argtypes = [ctypes.c_uint64]
        _lib = L
    return _lib


class OracleError(RuntimeError):
    def __init__(self, status, msg=""):
        super().__init__("oracle status %d %s" % (status, msg))
        self.status = status


class OracleWriter:
    """ParquetFile restated on the CPU (in-memory output)."""

    def __init__(self, schema, props=None):
        L = lib()
        self._schema, self._keep = make_schema(schema)
        self._props = props if props is not None else make_props()
        st = ctypes.c_int(0)
        self._h = L.kpwo_open(ctypes.byref(self._schema), ctypes.byref(self._props), ctypes.byref(st))
        if not self._h:
            raise OracleError(st.value, "open")

    def write(self, rec: bytes):
        st = lib().kpwo_write(self._h, rec, len(rec))
        if st:
            raise OracleError(st, "write")

    def write_batch(self, data, offsets):
        n = len(offsets) - 1
        nw = ctypes.c_uint64(0)
        st = lib().kpwo_write_batch(self._h, data.ctypes.data, offsets.ctypes.data, n, ctypes.byref(nw))
        return st, nw.value

    def write_until_full(self, data, offsets, max_file_size):
        n = len(offsets) - 1
        na = ctypes.c_uint64(0)
        full = ctypes.c_int(0)
        st = lib().kpwo_write_until_full(self._h, data.ctypes.data, offsets.ctypes.data, n, max_file_size,
                                         ctypes.byref(na), ctypes.byref(full))
        return st, na.value, bool(full.value)

    def data_size(self):
        return lib().kpwo_data_size(self._h)

    def num_records(self):
        return lib().kpwo_num_records(self._h)

    def num_row_groups(self):
        return lib().kpwo_num_row_groups(self._h)

    def close(self):
        st = lib().kpwo_close(self._h)
        if st:
            raise OracleError(st, "close")

    def file_bytes(self):
        p = ctypes.c_void_p()
        n = ctypes.c_uint64()
        st = lib().kpwo_file_bytes(self._h, ctypes.byref(p), ctypes.byref(n))
        if st:
            raise OracleError(st, "file_bytes")
        return (ctypes.c_char * n.value).from_address(p.value).raw if n.value else b""   # >= 2 GiB too

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().kpwo_free(h)
            self._h = None


def encode_file(schema, data, offsets, props=None):
    w = OracleWriter(schema, props)
    st, nw = w.write_batch(data, offsets)
    if st:
        raise OracleError(st, "write_batch at record %d" % nw)
    w.close()
    return w.file_bytes()


def rle_encode(values, bit_width):
    v = np.ascontiguousarray(values, dtype=np.uint32)
    cap = 16 + len(v) * 5 + 64
    out = np.zeros(cap, dtype=np.uint8)
    n = lib().kpwo_rle_encode(v.ctypes.data, len(v), bit_width, out.ctypes.data, cap)
    if n < 0:
        raise OracleError(-1, "rle")
    return bytes(out[:n])


def delta_encode(values, is_long):
    """DeltaBinaryPackingValuesWriterFor{Integer,Long}.getBytes() of a fresh writer."""
    v = np.ascontiguousarray(np.asarray(values).astype(np.int64).view(np.uint64))
    cap = 64 + len(v) * 10
    out = np.zeros(cap, dtype=np.uint8)
    n = lib().kpwo_delta_encode(v.ctypes.data, len(v), 1 if is_long else 0, out.ctypes.data, cap)
    if n < 0:
        raise OracleError(-1, "delta")
    return bytes(out[:n])


def snappy_compress(data: bytes):
    L = lib()
    cap = L.kpwo_snappy_max_compressed_length(len(data))
    out = ctypes.create_string_buffer(int(cap))
    n = L.kpwo_snappy_compress(data, len(data), out, cap)
    if n < 0:
        raise OracleError(-1, "snappy")
    return out.raw[:n]


def gzip_compress(data: bytes):
    """One page as CompressionCodecName.GZIP writes it (oracle_deflate.c)."""
    L = lib()
    cap = L.kpwo_gzip_bound(len(data))
    out = ctypes.create_string_buffer(int(cap))
    n = L.kpwo_gzip_compress(data, len(data), out, cap)
    if n < 0:
        raise OracleError(-1, "gzip")
    return out.raw[:n]


def deflate_raw(data: bytes):
    """zlib 1.2.11 level-6 raw deflate (windowBits -15, memLevel 8) of `data` (oracle_deflate.c)."""
    L = lib()
    cap = L.kpwo_gzip_bound(len(data))
    out = ctypes.create_string_buffer(int(cap))
    n = L.kpwo_deflate_raw(data, len(data), out, cap)
    if n < 0:
        raise OracleError(-1, "deflate")
    return out.raw[:n]
