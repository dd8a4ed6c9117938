"""kpw — MI355X-native Parquet column-chunk encoder for the Kafka->Parquet sink.

Host-side mirror of the reference seam (src/main/java/ir/sahab/kafka/reader/ParquetFile.java):
``ParquetFile`` / ``ParquetProperties`` with the same names, argument meaning and error
behaviour, backed by the HIP C-ABI library ``libkpw_gpu.so`` (include/kpw_gpu.h).  There
is no CPU fallback: constructing a ParquetFile without the library raises.
"""
from ._lib import (KpwError, InvalidProtoError, load_library, library_path, Schema, Column,
                   UNCOMPRESSED, SNAPPY, GZIP)
from .parquet_file import ParquetFile, ParquetProperties, pinned_empty
from .encoder import Encoder, DeviceBuffer

__all__ = ["ParquetFile", "ParquetProperties", "Encoder", "DeviceBuffer", "Schema", "Column", "KpwError", "InvalidProtoError",
           "load_library", "library_path", "UNCOMPRESSED", "SNAPPY", "GZIP", "pinned_empty"]
