"""ctypes binding of libkpw_gpu.so (include/kpw_gpu.h).  Fails loudly if missing."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)

UNCOMPRESSED, SNAPPY, GZIP = 0, 1, 2   # CompressionCodecName values the reference passes through (ParquetFile.java:45)
KPW_OK, KPW_ERR_INVALID_PROTO = 0, -3
STATUS_NAMES = {0: "OK", -1: "INVALID_ARG", -2: "UNSUPPORTED", -3: "INVALID_PROTO", -4: "IO", -5: "DEVICE",
                -6: "NOMEM", -7: "STATE", -8: "LIMIT"}


class KpwError(RuntimeError):
    """A non-zero kpw_status.  .retryable mirrors what tryUntilSucceeds would retry
    (IOException only, KafkaProtoParquetWriter.java:410-428)."""

    def __init__(self, status, message=""):
        super().__init__("%s (%d): %s" % (STATUS_NAMES.get(status, "?"), status, message))
        self.status = status
        self.retryable = status == -4


class InvalidProtoError(KpwError):
    """Mirrors the reference's IllegalStateException("Invalid proto message received.")
    (KafkaProtoParquetWriter.java:271-276)."""

    def __init__(self, status, message="", record=-1):
        super().__init__(status, message)
        self.record = record


class Column:
    def __init__(self, name, field_number, proto_type, label):
        self.name, self.field_number, self.proto_type, self.label = name, field_number, proto_type, label


class Schema:
    """A proto2 message as ProtoSchemaConverter sees it: top-level scalar fields in
    declaration order (descriptor.proto Type/Label numbering)."""

    def __init__(self, message_name, columns, proto_class=None):
        self.message_name = message_name
        self.columns = [c if isinstance(c, Column) else Column(*c) for c in columns]
        self.proto_class = proto_class or message_name


class _ColumnDesc(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("field_number", ctypes.c_int32),
                ("proto_type", ctypes.c_int32), ("label", ctypes.c_int32)]


class _SchemaC(ctypes.Structure):
    _fields_ = [("message_name", ctypes.c_char_p), ("proto_class", ctypes.c_char_p),
                ("num_columns", ctypes.c_int32), ("columns", ctypes.POINTER(_ColumnDesc))]


class _PropsC(ctypes.Structure):
    _fields_ = [("block_size", ctypes.c_int64), ("page_size", ctypes.c_int32),
                ("dictionary_page_size", ctypes.c_int32), ("enable_dictionary", ctypes.c_int32),
                ("codec", ctypes.c_int32), ("writer_version", ctypes.c_int32), ("reserved0", ctypes.c_int32),
                ("dfs_block_size", ctypes.c_int64), ("max_padding_size", ctypes.c_int64)]


class PageInfo(ctypes.Structure):
    _fields_ = [("page_type", ctypes.c_int32), ("num_values", ctypes.c_int32), ("encoding", ctypes.c_int32),
                ("dl_encoding", ctypes.c_int32), ("rl_encoding", ctypes.c_int32), ("has_stats", ctypes.c_int32),
                ("uncompressed_size", ctypes.c_int64), ("compressed_size", ctypes.c_int64),
                ("offset", ctypes.c_uint64), ("null_count", ctypes.c_int64), ("has_min_max", ctypes.c_int32),
                ("min_len", ctypes.c_int32), ("max_len", ctypes.c_int32), ("dl_byte_length", ctypes.c_int32),
                ("min_off", ctypes.c_uint64), ("max_off", ctypes.c_uint64), ("num_rows", ctypes.c_int32),
                ("rl_byte_length", ctypes.c_int32)]


class ChunkInfo(ctypes.Structure):
    _fields_ = [("column", ctypes.c_int32), ("first_page", ctypes.c_int32), ("num_pages", ctypes.c_int32),
                ("has_dictionary", ctypes.c_int32), ("num_values", ctypes.c_int64)]


class RowGroupInfo(ctypes.Structure):
    _fields_ = [("first_record", ctypes.c_int64), ("num_records", ctypes.c_int64),
                ("first_chunk", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class BatchInfo(ctypes.Structure):
    _fields_ = [("num_row_groups", ctypes.c_int32), ("num_chunks", ctypes.c_int32), ("num_pages", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("row_groups", ctypes.POINTER(RowGroupInfo)),
                ("chunks", ctypes.POINTER(ChunkInfo)), ("pages", ctypes.POINTER(PageInfo)),
                ("stats_bytes", ctypes.c_void_p), ("stats_len", ctypes.c_uint64),
                ("device_pages", ctypes.c_void_p), ("device_pages_len", ctypes.c_uint64),
                ("records_consumed", ctypes.c_int64), ("open_records", ctypes.c_int64),
                ("open_buffered_size", ctypes.c_int64), ("invalid_record", ctypes.c_int64)]


def make_schema(schema):
    cols = (_ColumnDesc * len(schema.columns))()
    keep = [cols]
    for i, c in enumerate(schema.columns):
        b = c.name.encode()
        keep.append(b)
        cols[i] = _ColumnDesc(b, c.field_number, c.proto_type, c.label)
    mn, pc = schema.message_name.encode(), schema.proto_class.encode()
    keep += [mn, pc]
    return _SchemaC(mn, pc, len(schema.columns), cols), keep


def library_path():
    return os.environ.get("KPW_GPU_LIB", os.path.join(_PKG, "libkpw_gpu.so"))


_lib = None


def load_library():
    """Load libkpw_gpu.so; raises (no CPU fallback) if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if not os.path.exists(path):
        raise KpwError(-5, "libkpw_gpu.so not found at %s: build it with `make -C kafka-parquet-writer_amd` "
                           "(there is deliberately no CPU fallback)" % path)
    L = ctypes.CDLL(path)
    vp, u64, i64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int
    L.kpw_writer_open.restype = vp
    L.kpw_writer_open.argtypes = [i32, ctypes.POINTER(_SchemaC), ctypes.POINTER(_PropsC), ctypes.c_char_p,
                                  ctypes.POINTER(i32)]
    L.kpw_writer_write.argtypes = [vp, vp, vp, u64]
    L.kpw_writer_write_async.argtypes = [vp, vp, vp, u64]
    L.kpw_writer_write_until_full.argtypes = [vp, vp, vp, u64, i64, ctypes.POINTER(u64), ctypes.POINTER(i32)]
    L.kpw_writer_data_size.restype = i64
    L.kpw_writer_data_size.argtypes = [vp]
    L.kpw_writer_num_records.restype = i64
    L.kpw_writer_num_records.argtypes = [vp]
    L.kpw_writer_creation_time_ms.restype = i64
    L.kpw_writer_creation_time_ms.argtypes = [vp]
    L.kpw_writer_close.argtypes = [vp]
    L.kpw_writer_file_bytes.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(u64)]
    L.kpw_writer_failed_record.restype = i64
    L.kpw_writer_failed_record.argtypes = [vp]
    L.kpw_writer_last_error.restype = ctypes.c_char_p
    L.kpw_writer_last_error.argtypes = [vp]
    L.kpw_writer_free.argtypes = [vp]
    L.kpw_encoder_create.restype = vp
    L.kpw_encoder_create.argtypes = [i32, ctypes.POINTER(_SchemaC), ctypes.POINTER(_PropsC), ctypes.POINTER(i32)]
    L.kpw_encoder_destroy.argtypes = [vp]
    L.kpw_encoder_last_error.restype = ctypes.c_char_p
    L.kpw_encoder_last_error.argtypes = [vp]
    L.kpw_encoder_encode.argtypes = [vp, vp, vp, u64, i32, i64, vp, ctypes.POINTER(BatchInfo)]
    L.kpw_encoder_copy_pages.argtypes = [vp, u64, u64, vp]
    L.kpw_encoder_stage_times.argtypes = [vp, ctypes.POINTER(ctypes.c_float), i32]
    L.kpw_writer_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_double), i32]
    L.kpw_host_alloc.restype = vp
    L.kpw_host_alloc.argtypes = [u64, ctypes.POINTER(i32)]
    L.kpw_host_free.argtypes = [vp]
    L.kpw_trim_caches.argtypes = []
    L.kpw_trim_caches.restype = None
    L.kpw_cache_stats.argtypes = [ctypes.POINTER(ctypes.c_double), i32]
    L.kpw_device_alloc.restype = vp
    L.kpw_device_alloc.argtypes = [i32, u64, ctypes.POINTER(i32)]
    L.kpw_device_free.argtypes = [vp]
    L.kpw_device_free.restype = None
    L.kpw_copy_h2d.argtypes = [i32, vp, vp, u64]
    L.kpw_copy_d2h.argtypes = [i32, vp, vp, u64]
    _lib = L
    return L


EXPORTED = ["kpw_writer_open", "kpw_writer_write", "kpw_writer_write_async", "kpw_writer_write_until_full", "kpw_writer_data_size",
            "kpw_writer_num_records", "kpw_writer_creation_time_ms", "kpw_writer_close", "kpw_writer_file_bytes",
            "kpw_writer_failed_record", "kpw_writer_last_error", "kpw_writer_free", "kpw_encoder_create",
            "kpw_encoder_destroy", "kpw_encoder_last_error", "kpw_encoder_encode", "kpw_encoder_copy_pages",
            "kpw_encoder_stage_times", "kpw_host_alloc", "kpw_host_free", "kpw_writer_stats", "kpw_trim_caches",
            "kpw_cache_stats", "kpw_device_alloc", "kpw_device_free", "kpw_copy_h2d", "kpw_copy_d2h"]


CACHE_STATS = ["dev_cache_cap", "pin_cache_cap", "dev_live", "dev_idle", "pin_live", "pin_idle", "dev_malloc_n",
               "dev_malloc_ms", "dev_free_n", "dev_free_ms", "pin_malloc_n", "pin_malloc_ms", "pin_free_n",
               "pin_free_ms", "dev_hits", "pin_hits", "dev_retry", "dev_sync_n", "dev_sync_ms",
               "gate_admits", "gate_wait_ms"]


def cache_stats():
    """kpw_cache_stats as a dict (process-wide allocator figures, include/kpw_gpu.h)."""
    L = load_library()
    buf = (ctypes.c_double * len(CACHE_STATS))()
    k = L.kpw_cache_stats(buf, len(CACHE_STATS))
    return {name: buf[i] for i, name in enumerate(CACHE_STATS[:k])}
