"""Encoder — the flush-path primitive (kpw_encoder_*): device-resident record batch ->
encoded pages + metadata for every row group parquet-mr would cut.  Used by bench.py and
the GPU parity tests; batches live in DeviceBuffer memory (kpw_device_alloc: the library's own
HIP runtime, so no second runtime is involved)."""
import ctypes

import numpy as np

from ._lib import KpwError, load_library, make_schema, _PropsC, BatchInfo

MiB = 1024 * 1024


def props_c(block_size=128 * MiB, page_size=128 * MiB, codec=0, enable_dictionary=True, dictionary_page_size=MiB,
            writer_version=1):
    return _PropsC(block_size, page_size, dictionary_page_size, 1 if enable_dictionary else 0, codec, writer_version, 0, 0,
                   8 * MiB)


class DeviceBuffer:
    """HBM owned by libkpw_gpu.so (kpw_device_alloc); `ptr` is the device address.
    DeviceBuffer(nbytes) or DeviceBuffer.from_array(numpy array) (a synchronous H2D copy)."""

    def __init__(self, nbytes, device=0):
        self._L = load_library()
        self.device = device
        self.nbytes = int(nbytes)
        st = ctypes.c_int(0)
        self.ptr = self._L.kpw_device_alloc(device, max(1, self.nbytes), ctypes.byref(st))
        if not self.ptr:
            raise KpwError(st.value, "device allocation of %d bytes" % self.nbytes)

    @classmethod
    def from_array(cls, arr, device=0):
        a = np.ascontiguousarray(arr)
        b = cls(a.nbytes, device)
        if a.nbytes:
            st = b._L.kpw_copy_h2d(device, b.ptr, a.ctypes.data, a.nbytes)
            if st:
                raise KpwError(st, "H2D copy")
        return b

    def to_array(self, dtype=np.uint8, count=None):
        dt = np.dtype(dtype)
        n = self.nbytes // dt.itemsize if count is None else count
        out = np.empty(max(1, n), dtype=dt)
        if n:
            st = self._L.kpw_copy_d2h(self.device, out.ctypes.data, self.ptr, n * dt.itemsize)
            if st:
                raise KpwError(st, "D2H copy")
        return out[:n]

    def free(self):
        if getattr(self, "ptr", None):
            self._L.kpw_device_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.free()


class Encoder:
    def __init__(self, schema, device=0, **props):
        self._L = load_library()
        self._schema_c, self._keep = make_schema(schema)
        self._props = props_c(**props)
        st = ctypes.c_int(0)
        self._h = self._L.kpw_encoder_create(device, ctypes.byref(self._schema_c), ctypes.byref(self._props),
                                             ctypes.byref(st))
        if not self._h:
            raise KpwError(st.value, "encoder create")
        self.info = BatchInfo()

    def encode(self, d_data_ptr, d_offsets_ptr, n, final=True, stream=None):
        st = self._L.kpw_encoder_encode(self._h, d_data_ptr, d_offsets_ptr, n, 1 if final else 0, 0,
                                        stream, ctypes.byref(self.info))
        if st:
            raise KpwError(st, (self._L.kpw_encoder_last_error(self._h) or b"").decode(errors="replace"))
        return self.info

    def stage_times(self):
        arr = (ctypes.c_float * 10)()
        n = self._L.kpw_encoder_stage_times(self._h, arr, 10)
        return list(arr[:n])

    def pages_bytes(self):
        n = self.info.device_pages_len
        out = np.empty(max(1, n), dtype=np.uint8)
        if n:
            st = self._L.kpw_encoder_copy_pages(self._h, 0, n, out.ctypes.data)
            if st:
                raise KpwError(st, "copy_pages")
        return out[:n].tobytes()

    def row_groups(self):
        i = self.info
        return [(i.row_groups[k].first_record, i.row_groups[k].num_records) for k in range(i.num_row_groups)]

    def pages(self):
        i = self.info
        stats = ctypes.string_at(i.stats_bytes, i.stats_len) if i.stats_len else b""
        out = []
        for k in range(i.num_pages):
            p = i.pages[k]
            out.append(dict(page_type=p.page_type, num_values=p.num_values, encoding=p.encoding,
                            dl_encoding=p.dl_encoding, uncompressed_size=p.uncompressed_size,
                            compressed_size=p.compressed_size, offset=p.offset, null_count=p.null_count,
                            has_min_max=p.has_min_max, min=stats[p.min_off:p.min_off + p.min_len],
                            max=stats[p.max_off:p.max_off + p.max_len], dl_byte_length=p.dl_byte_length, rl_byte_length=p.rl_byte_length,
                            num_rows=p.num_rows))
        return out

    def chunks(self):
        i = self.info
        return [dict(column=i.chunks[k].column, first_page=i.chunks[k].first_page, num_pages=i.chunks[k].num_pages,
                     has_dictionary=i.chunks[k].has_dictionary, num_values=i.chunks[k].num_values)
                for k in range(i.num_chunks)]

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.kpw_encoder_destroy(h)
            self._h = None
