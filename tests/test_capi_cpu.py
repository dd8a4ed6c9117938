"""CPU-side checks of the C-ABI library: it builds for gfx950, loads, exports every
symbol include/kpw_gpu.h declares, and rejects bad arguments before touching a GPU."""
import ctypes
import os
import re

import pytest

import kpw
from kpw import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_header_symbols():
    L = kpw.load_library()
    hdr = open(os.path.join(ROOT, "include", "kpw_gpu.h")).read()
    declared = set(re.findall(r"\b(kpw_[a-z0-9_]+)\s*\(", hdr))
    assert declared == set(_lib.EXPORTED)
    for sym in declared:
        assert hasattr(L, sym), sym


def test_gfx950_code_object_present():
    data = open(kpw.library_path(), "rb").read()
    assert b"gfx950" in data


def _schema(cols):
    return kpw.Schema("T", cols)


def test_create_rejects_bad_schema_without_gpu():
    L = kpw.load_library()
    st = ctypes.c_int(0)
    # enum field (proto type 14): outside the accelerated path
    sc, keep = _lib.make_schema(_schema([("e", 1, 14, 2)]))
    pr = kpw.encoder.props_c()
    h = L.kpw_encoder_create(0, ctypes.byref(sc), ctypes.byref(pr), ctypes.byref(st))
    assert not h and st.value == -2
    # repeated label
    sc, keep = _lib.make_schema(_schema([("r", 1, 5, 3)]))
    h = L.kpw_encoder_create(0, ctypes.byref(sc), ctypes.byref(pr), ctypes.byref(st))
    assert not h and st.value == -2
    # null schema
    h = L.kpw_encoder_create(0, None, ctypes.byref(pr), ctypes.byref(st))
    assert not h and st.value == -1
    # PARQUET_2_0 is an explicit opt-in and needs the dictionary on (the reference cannot
    # turn it off); unknown writer versions are rejected
    sc, keep = _lib.make_schema(_schema([("a", 1, 5, 2)]))
    pr2 = kpw.encoder.props_c(writer_version=2, enable_dictionary=False)
    h = L.kpw_encoder_create(0, ctypes.byref(sc), ctypes.byref(pr2), ctypes.byref(st))
    assert not h and st.value == -2
    pr3 = kpw.encoder.props_c(writer_version=3)
    h = L.kpw_encoder_create(0, ctypes.byref(sc), ctypes.byref(pr3), ctypes.byref(st))
    assert not h and st.value == -2


def test_page_info_layout():
    """kpw_page_info as declared in include/kpw_gpu.h (the ctypes mirror must match it)."""
    assert ctypes.sizeof(_lib.PageInfo) == 96
    assert _lib.PageInfo.min_off.offset == 72 and _lib.PageInfo.num_rows.offset == 88


def test_null_handles():
    L = kpw.load_library()
    assert L.kpw_writer_write(None, None, None, 0) == -1
    assert L.kpw_writer_close(None) == -1
    assert L.kpw_writer_data_size(None) == -1
    assert L.kpw_encoder_encode(None, None, None, 0, 1, 0, None, None) == -1


def test_properties_dictionary_quirk():
    """ParquetFile.java:48-50 + parquet-mr 1.10.1 builder default: dictionary stays on."""
    p = kpw.ParquetProperties(enable_dictionary=False)
    assert p.to_c().enable_dictionary == 1
    assert p.to_c().page_size == 128 * 1024 * 1024  # reference default pageSize (KPW:473-474)


def test_properties_hdfs_alignment():
    """fs.defaultFS on a block file system selects PaddingAlignment (HadoopOutputFile
    BLOCK_FS_SCHEMES) with dfs.blocksize (Configuration.getLongBytes suffixes) and 8 MiB max
    padding; a local file system NoAlignment (dfs_block_size 0)."""
    MiB = 1 << 20
    p = kpw.ParquetProperties(hadoop_conf={"fs.defaultFS": "hdfs://nn:8020"})
    assert (p.dfs_block_size, p.max_padding_size) == (128 * MiB, 8 * MiB)
    p = kpw.ParquetProperties(hadoop_conf={"fs.defaultFS": "viewfs://c", "dfs.blocksize": "256m"})
    assert p.dfs_block_size == 256 * MiB and p.to_c().dfs_block_size == 256 * MiB
    p = kpw.ParquetProperties(hadoop_conf={"fs.defaultFS": "file:///", "dfs.blocksize": "256m"})
    assert p.dfs_block_size == 0 and p.to_c().dfs_block_size == 0
    p = kpw.ParquetProperties(dfs_block_size=3 * MiB, max_padding_size=MiB)
    c = p.to_c()
    assert (c.dfs_block_size, c.max_padding_size) == (3 * MiB, MiB)


def test_properties_alignment_follows_resolved_target_path():
    """targetDir = new Path(fs.defaultFS, builder.targetDir) (KafkaProtoParquetWriter.java:137-141):
    a target dir with its own scheme decides the file system, otherwise fs.defaultFS does."""
    from kpw.parquet_file import resolved_scheme
    MiB = 1 << 20
    assert resolved_scheme("hdfs://nn:8020", "/data/out") == "hdfs"
    assert resolved_scheme("hdfs://nn:8020", "file:///data/out") == "file"
    assert resolved_scheme("file:///", "webhdfs://nn/x") == "webhdfs"
    p = kpw.ParquetProperties(hadoop_conf={"fs.defaultFS": "hdfs://nn:8020"}, target_dir="file:///tmp/out")
    assert p.dfs_block_size == 0
    p = kpw.ParquetProperties(hadoop_conf={"fs.defaultFS": "file:///"}, target_dir="hdfs://nn/out")
    assert p.dfs_block_size == 128 * MiB
    p = kpw.ParquetProperties(hadoop_conf={"fs.defaultFS": "hdfs://nn:8020"}, target_dir="/rel/out")
    assert p.dfs_block_size == 128 * MiB


def test_par_copy_covers_every_byte():
    """The host staging copy (kpw::par_copy, writer slots and file assembly) splits large copies
    over threads; every byte must arrive whatever n % threads is (a chunk size of floor(n/t)
    rounded to 4 KiB once dropped the last n % t bytes: 6 stale bytes in a C4 slot)."""
    import numpy as np
    L = kpw.load_library()
    fn = getattr(L, "_ZN3kpw8par_copyEPhPKhm")
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    fn.restype = None
    rng = np.random.default_rng(5)
    src = rng.integers(0, 256, 40 << 20, dtype=np.uint8)
    for n in (32600070, 7 * 4657152 + 1, 8 * (4 << 20) + 3, 5 * 4096 * 1024 + 4, (4 << 20) * 3 - 1, 12345, 40 << 20):
        dst = np.zeros(n + 16, dtype=np.uint8)
        fn(dst.ctypes.data, src.ctypes.data, n)
        assert np.array_equal(dst[:n], src[:n]), n
        assert not dst[n:].any(), n
