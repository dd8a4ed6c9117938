"""ParquetFile / ParquetProperties — host-side mirror of the reference seam.

Reference: src/main/java/ir/sahab/kafka/reader/ParquetFile.java
  ParquetFile(Path filePath, Class<T> protoClass, ParquetProperties properties)   :36-54
  write(T record) throws IOException                                            :59-62
  close() throws IOException                                                    :65-68
  getCreationDate()                                                             :70-72
  getDataSize()                                                                 :77-79
  getNumWrittenRecords()                                                        :81-83
  ParquetProperties(hadoopConf, blockSize, compressionCodecName, pageSize,
                    enableDictionary)                                           :105-122

Differences forced by the GPU boundary: write() takes the serialized record value
(record.value(), KafkaProtoParquetWriter.java:270) instead of a parsed T — parsing is
kernel K1 — and write_batch() accepts many values at once.  An invalid value raises
InvalidProtoError, the reference's IllegalStateException path (KPW:271-276); records
before it stay written, it and the records after it are not.  Writes of <= 65536 records
(the reference's one-record loop) raise it from that write, like parseFrom; a larger
write is validated on the GPU and the error is raised by the next call (write,
get_data_size or close), when get_num_written_records() is also corrected.
Instances are not thread-safe (ParquetFile.java:19-20); separate instances may be used
from separate threads (one writer per worker thread, KafkaProtoParquetWriter.java:175-179).
"""
import ctypes
import datetime

import numpy as np

from ._lib import (KpwError, InvalidProtoError, load_library, make_schema, _PropsC, UNCOMPRESSED, SNAPPY, GZIP,
                   KPW_ERR_INVALID_PROTO)

MiB = 1024 * 1024


HDFS_SCHEMES = ("hdfs", "webhdfs", "viewfs")   # parquet-mr 1.10.1 HadoopOutputFile.BLOCK_FS_SCHEMES


class ParquetProperties:
    """ParquetFile.ParquetProperties (ParquetFile.java:105-122).

    The output stream itself is a local path or memory.  hadoop_conf (a dict of Hadoop
    configuration keys) only selects parquet-mr's row-group alignment: when the file's path is
    on a block file system ParquetFileWriter uses PaddingAlignment with the file system's block
    size (dfs.blocksize, default 128 MiB) and ParquetWriter's MAX_PADDING_SIZE_DEFAULT (8 MiB):
    row groups are sized to end at HDFS block boundaries and zero padding fills a block's last
    <= 8 MiB.  The reference writes under targetDir = new Path(fs.defaultFS, builder.targetDir)
    (KafkaProtoParquetWriter.java:137-141), so the file system is the resolved path's: a
    target_dir with its own scheme ("file:///data") wins over fs.defaultFS, as in Hadoop's
    Path(parent, child).  dfs_block_size / max_padding_size set the same explicitly (0 =
    NoAlignment, a local file system).  Byte parity of padded files with parquet-mr is checked
    against the oracle only (the reference holds no padded fixture): parity unpinned."""

    def __init__(self, hadoop_conf=None, block_size=128 * MiB, compression_codec_name=UNCOMPRESSED,
                 page_size=128 * MiB, enable_dictionary=True, writer_version=1, dfs_block_size=None,
                 max_padding_size=8 * MiB, target_dir=None):
        self.hadoop_conf = hadoop_conf
        self.block_size = int(block_size)
        self.compression_codec_name = int(compression_codec_name)
        self.page_size = int(page_size)
        self.enable_dictionary = bool(enable_dictionary)
        # ParquetFile.java:42-50 never sets a writer version (PARQUET_1_0); 2 = PARQUET_2_0,
        # an explicit opt-in beyond the reference (DataPageV2 + DELTA fallback encodings)
        self.writer_version = int(writer_version)
        if dfs_block_size is None:
            dfs_block_size = 0
            conf = hadoop_conf if isinstance(hadoop_conf, dict) else {}
            scheme = resolved_scheme(str(conf.get("fs.defaultFS", "")), target_dir)
            if scheme in HDFS_SCHEMES:
                dfs_block_size = _hadoop_size(conf.get("dfs.blocksize", 128 * MiB))
        self.dfs_block_size = int(dfs_block_size)
        self.max_padding_size = int(max_padding_size)

    def to_c(self):
        # ParquetFile.java:48-50 only ever calls enableDictionaryEncoding(); parquet-mr 1.10.1's
        # builder defaults dictionary encoding to ON, so the reference writes dictionaries
        # even when enableDictionary is false.  Reproduced here on purpose.
        effective_dictionary = 1
        return _PropsC(self.block_size, self.page_size, MiB, effective_dictionary, self.compression_codec_name,
                       self.writer_version, 0, self.dfs_block_size, self.max_padding_size)


def resolved_scheme(default_fs, target_dir=None):
    """Scheme of new Path(default_fs, target_dir) (org.apache.hadoop.fs.Path(Path, Path)): the
    child's scheme when it has one, otherwise the parent's."""
    def scheme(u):
        u = str(u or "")
        head = u.split("/", 1)[0]
        return head[:-1].lower() if head.endswith(":") and len(head) > 2 else ""
    return scheme(target_dir) or scheme(default_fs)


def _hadoop_size(v):
    """Configuration.getLongBytes: a number with an optional k/m/g/t/p/e suffix (binary)."""
    if isinstance(v, (int, float)):
        return int(v)
    t = str(v).strip().lower()
    mult = {"k": 1 << 10, "m": 1 << 20, "g": 1 << 30, "t": 1 << 40, "p": 1 << 50, "e": 1 << 60}
    if t and t[-1] in mult:
        return int(t[:-1]) * mult[t[-1]]
    return int(t)


def _as_batch(values):
    if isinstance(values, tuple) and len(values) == 2:
        data, offsets = values
        return np.ascontiguousarray(data, dtype=np.uint8), np.ascontiguousarray(offsets, dtype=np.uint64)
    values = list(values)
    offsets = np.zeros(len(values) + 1, dtype=np.uint64)
    if values:
        np.cumsum([len(v) for v in values], out=offsets[1:])
    data = np.frombuffer(b"".join(values), dtype=np.uint8) if values else np.zeros(1, np.uint8)
    return np.ascontiguousarray(data), offsets


def pinned_empty(nbytes):
    """A numpy uint8 array in pinned host memory (kpw_host_alloc): record batches placed here
    are DMA'd to the GPU by write_batch without a host copy (north_star: polled batches land
    in pinned staging buffers).  Freed with the array."""
    import weakref
    L = load_library()
    st = ctypes.c_int(0)
    p = L.kpw_host_alloc(max(1, int(nbytes)), ctypes.byref(st))
    if not p:
        raise KpwError(st.value, "kpw_host_alloc(%d)" % nbytes)
    # views of the array keep it (their .base) alive, so the memory outlives every view
    arr = np.ctypeslib.as_array((ctypes.c_uint8 * max(1, int(nbytes))).from_address(p))
    weakref.finalize(arr, L.kpw_host_free, p)
    return arr


class ParquetFile:
    """A Parquet file of proto messages, encoded on an MI355X (HIP C-ABI)."""

    def __init__(self, file_path, proto_schema, properties=None, device=0):
        self._L = load_library()
        self.file_path = file_path
        self.proto_schema = proto_schema
        self._props = properties or ParquetProperties()
        self._schema_c, self._keep = make_schema(proto_schema)
        pc = self._props.to_c()
        st = ctypes.c_int(0)
        path = file_path.encode() if isinstance(file_path, str) else file_path
        self._h = self._L.kpw_writer_open(device, ctypes.byref(self._schema_c), ctypes.byref(pc), path, ctypes.byref(st))
        if not self._h:
            raise KpwError(st.value, "ParquetFile open")
        self._creation = datetime.datetime.now()

    def _check(self, st, what):
        if st == 0:
            return
        msg = (self._L.kpw_writer_last_error(self._h) or b"").decode(errors="replace")
        if st == KPW_ERR_INVALID_PROTO:
            raise InvalidProtoError(st, msg, self._L.kpw_writer_failed_record(self._h))
        raise KpwError(st, "%s: %s" % (what, msg))

    def write(self, record_value: bytes):
        """ParquetFile.write(T) for one serialized record value."""
        self.write_batch([record_value])

    def write_batch(self, values):
        """values: list of bytes, or (data uint8[], offsets uint64[n+1])."""
        data, offsets = _as_batch(values)
        n = len(offsets) - 1
        self._check(self._L.kpw_writer_write(self._h, data.ctypes.data, offsets.ctypes.data, n), "write")

    def write_batch_async(self, data, offsets):
        """kpw_writer_write_async: `data` (a pinned_empty batch) may still be read by the DMA
        until the next call on this file returns; `offsets` may be reused at once."""
        n = len(offsets) - 1
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        self._check(self._L.kpw_writer_write_async(self._h, data.ctypes.data, offsets.ctypes.data, n), "write")

    def write_until_full(self, values, max_file_size):
        data, offsets = _as_batch(values)
        n = len(offsets) - 1
        na = ctypes.c_uint64(0)
        full = ctypes.c_int(0)
        self._check(self._L.kpw_writer_write_until_full(self._h, data.ctypes.data, offsets.ctypes.data, n,
                                                        max_file_size, ctypes.byref(na), ctypes.byref(full)),
                    "write_until_full")
        return na.value, bool(full.value)

    def get_data_size(self):
        v = self._L.kpw_writer_data_size(self._h)
        if v < 0:
            self._check(KPW_ERR_INVALID_PROTO if self._L.kpw_writer_failed_record(self._h) >= 0 else -5, "getDataSize")
        return v

    def get_num_written_records(self):
        return self._L.kpw_writer_num_records(self._h)

    def get_creation_date(self):
        return self._creation

    def close(self):
        self._check(self._L.kpw_writer_close(self._h), "close")

    def pipeline_stats(self):
        """kpw_writer_stats: accumulated job / byte counts and per-stage device ms."""
        arr = (ctypes.c_double * 18)()
        n = self._L.kpw_writer_stats(self._h, arr, 18)
        names = ["jobs", "records", "record_bytes", "page_bytes_uncompressed", "page_bytes_compressed",
                 "decode_ms", "plan_ms", "stats_dict_ms", "rle_ms", "layout_plain_write_ms", "compress_ms",
                 "metadata_ms", "total_ms", "k_decode_ms", "k7_snappy_ms", "worker_encode_wall_ms", "lookback_fallbacks", "h2d_span_ms"]
        return dict(zip(names, list(arr[:n])))

    def file_bytes(self):
        p = ctypes.c_void_p()
        n = ctypes.c_uint64()
        self._check(self._L.kpw_writer_file_bytes(self._h, ctypes.byref(p), ctypes.byref(n)), "file_bytes")
        # (ctypes.string_at takes a C int size: files of >= 2 GiB need the array view)
        return (ctypes.c_char * n.value).from_address(p.value).raw if n.value else b""

    # AutoCloseable
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.kpw_writer_free(h)
            self._h = None

    # reference-style camelCase aliases
    getDataSize = get_data_size
    getNumWrittenRecords = get_num_written_records
    getCreationDate = get_creation_date
