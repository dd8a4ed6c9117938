"""Helpers for the GPU parity tests: run the HIP encoder on device-resident batches and
compare, page by page, with the CPU oracle's file for the same records and properties."""
import io
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import oracle
import pqwalk

MiB = 1024 * 1024


def to_device(data, offsets):
    """Record bytes and u64 offsets in HBM allocated by the library itself (kpw.DeviceBuffer):
    one HIP runtime owns every device pointer the encoder sees."""
    import kpw
    d = kpw.DeviceBuffer.from_array(np.ascontiguousarray(data) if len(data) else np.zeros(1, np.uint8))
    o = kpw.DeviceBuffer.from_array(np.ascontiguousarray(offsets, dtype=np.uint64))
    return d, o


def gpu_encoder_pages(schema, data, offsets, codec=0, block_size=128 * MiB, page_size=128 * MiB, dictionary=True,
                      writer_version=1, enc=None, dict_page_size=MiB):
    """Returns (row_groups, [(rg, col, [page dicts with 'body'])]) from the HIP encoder
    (a fresh one, or `enc` to reuse an encoder across batches)."""
    import kpw
    if enc is None:
        enc = kpw.Encoder(kpw.Schema(schema.message_name, schema.columns, schema.proto_class), codec=codec,
                          block_size=block_size, page_size=page_size, enable_dictionary=dictionary,
                          writer_version=writer_version, dictionary_page_size=dict_page_size)
    d, o = to_device(data, offsets)
    info = enc.encode(d.ptr, o.ptr, len(offsets) - 1, final=True)
    blob = enc.pages_bytes()
    pages = enc.pages()
    chunks = enc.chunks()
    rgs = enc.row_groups()
    out = []
    ncols = len(schema.columns)
    for ci, ch in enumerate(chunks):
        pl = []
        for p in pages[ch["first_page"]:ch["first_page"] + ch["num_pages"]]:
            q = dict(p)
            q["body"] = blob[p["offset"]:p["offset"] + p["compressed_size"]]
            pl.append(q)
        out.append((ci // ncols, ch["column"], pl))
    return rgs, out, info, enc


def oracle_pages(fb):
    """Group oracle file pages by (rg, col)."""
    res = {}
    for pg in pqwalk.pages(fb):
        res.setdefault((pg["rg"], pg["col"]), []).append(pg)
    return res


def oracle_row_groups(fb):
    fm = pqwalk.footer(fb)
    out, start = [], 0
    for rg in fm[4]:
        out.append((start, rg[3]))
        start += rg[3]
    return out


def oracle_props(**kw):
    return oracle.make_props(block_size=kw.get("block_size", 128 * MiB), page_size=kw.get("page_size", 128 * MiB),
                             codec=kw.get("codec", 0), enable_dictionary=kw.get("dictionary", True),
                             writer_version=kw.get("writer_version", 1), dictionary_page_size=kw.get("dict_page_size", MiB))


def compare_pages(schema, data, offsets, **kw):
    """Returns a list of human-readable mismatches (empty = byte-identical pages)."""
    fb = oracle.encode_file(schema, data, offsets, oracle_props(**kw))
    return compare_to_file(schema, data, offsets, fb, **kw)[0]


def compare_to_file(schema, data, offsets, fb, **kw):
    """HIP encoder pages of the batch vs the pages of the oracle file `fb`.
    Returns (mismatches, batch info)."""
    rgs, gpages, info, enc = gpu_encoder_pages(schema, data, offsets, **kw)
    errs = []
    orgs = oracle_row_groups(fb)
    if [tuple(r) for r in rgs] != [tuple(r) for r in orgs]:
        errs.append("row groups differ: gpu %r oracle %r" % (rgs[:8], orgs[:8]))
        return errs, info
    op = oracle_pages(fb)
    for rg, col, pl in gpages:
        ol = op.get((rg, col), [])
        name = schema.columns[col][0]
        if len(ol) != len(pl):
            errs.append("rg %d col %s: page count gpu %d oracle %d" % (rg, name, len(pl), len(ol)))
            continue
        for k, (g, o) in enumerate(zip(pl, ol)):
            h = o["header"]
            ptype = h[1]
            if g["page_type"] != ptype:
                errs.append("rg %d col %s page %d: type gpu %d oracle %d" % (rg, name, k, g["page_type"], ptype))
                continue
            if g["uncompressed_size"] != h[2] or g["compressed_size"] != h[3]:
                errs.append("rg %d col %s page %d: sizes gpu (%d,%d) oracle (%d,%d)" % (
                    rg, name, k, g["uncompressed_size"], g["compressed_size"], h[2], h[3]))
            if ptype in (0, 3):
                if ptype == 0:
                    dh = h[5]
                    got, want = (g["num_values"], g["encoding"], g["dl_encoding"]), (dh[1], dh[2], dh[3])
                    st = dh.get(5, {})
                else:   # DataPageHeaderV2
                    dh = h[8]
                    got = (g["num_values"], g["null_count"], g["num_rows"], g["encoding"], g["dl_byte_length"],
                           g["rl_byte_length"])
                    want = (dh[1], dh[2], dh[3], dh[4], dh[5], dh[6])
                    st = dh.get(8, {})
                if got != want:
                    errs.append("rg %d col %s page %d: header gpu %r oracle %r" % (rg, name, k, got, want))
                if st.get(3, None) is not None and st.get(3) != g["null_count"]:
                    errs.append("rg %d col %s: null_count gpu %d oracle %d" % (rg, name, g["null_count"], st.get(3)))
                if 6 in st and (st[6] != g["min"] or st[5] != g["max"]):
                    errs.append("rg %d col %s: min/max gpu %r/%r oracle %r/%r" % (rg, name, g["min"][:20], g["max"][:20],
                                                                                st[6][:20], st[5][:20]))
            else:
                if (g["num_values"], g["encoding"]) != (h[7][1], h[7][2]):
                    errs.append("rg %d col %s dict page (entries, encoding) gpu %r oracle %r" % (
                        rg, name, (g["num_values"], g["encoding"]), (h[7][1], h[7][2])))
            if g["body"] != o["body"]:
                a, b = g["body"], o["body"]
                i = next((j for j in range(min(len(a), len(b))) if a[j] != b[j]), min(len(a), len(b)))
                errs.append("rg %d col %s page %d type %d: body differs at byte %d (len gpu %d oracle %d): gpu %s oracle %s" % (
                    rg, name, k, ptype, i, len(a), len(b), a[max(0, i - 8):i + 16].hex(), b[max(0, i - 8):i + 16].hex()))
    return errs, info


def gpu_file(schema, data, offsets, props=None, batches=1):
    """Full file through the ParquetFile drop-in (kpw_writer_*), in memory."""
    import kpw
    pf = kpw.ParquetFile(None, kpw.Schema(schema.message_name, schema.columns, schema.proto_class), props)
    n = len(offsets) - 1
    step = max(1, (n + batches - 1) // batches)
    for i in range(0, n, step):
        j = min(n, i + step)
        sub = offsets[i:j + 1] - offsets[i]
        pf.write_batch((data[int(offsets[i]):int(offsets[j])], sub))
    pf.close()
    return pf.file_bytes()


# ---------------------------------------------------------------- full-size parity, row group by row group

AHEAD = 10_001   # MAXIMUM_RECORD_COUNT_FOR_CHECK + 1: the next size check is at most this far


def _workers():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 8
    return max(1, min(16, n, int(os.environ.get("OMP_NUM_THREADS", "16"))))


def chunk_table(fb):
    """Per row group: (num_rows, [(chunk bytes, ColumnMetaData without file offsets)])."""
    fm = pqwalk.footer(fb)
    out = []
    for rg in fm[4]:
        cols = []
        for cc in rg[1]:
            md = dict(cc[3])
            start = min(md[9], md[11]) if md.get(11) else md[9]
            body = fb[start:start + md[7]]
            for k in (9, 10, 11):
                md.pop(k, None)
            cols.append((body, md))
        out.append((rg[3], cols))
    return out


def check_row_groups(schema, data, offs, fb, props):
    """Every row group of file `fb` (records data/offs) against the oracle, in parallel:
    parquet-mr's row groups are independent (after a flush InternalParquetRecordWriter resets
    recordCount and checks again at 100 records; column chunks depend only on their row
    group's records), so row group r is checked against the oracle run on records
    [start_r, end_r + AHEAD): its first row group must end at end_r (the cut is re-derived)
    and every column chunk must be byte-identical, with equal ColumnMetaData apart from file
    offsets.  Returns a list of mismatch descriptions (empty = identical)."""
    n = len(offs) - 1
    got = chunk_table(fb)
    starts = np.cumsum([0] + [r[0] for r in got])
    errs = []
    if starts[-1] != n:
        return ["row groups cover %d of %d records" % (starts[-1], n)]

    def one(r):
        s, cnt = int(starts[r]), got[r][0]
        e = min(n, s + cnt + AHEAD)
        w = oracle.OracleWriter(schema, props)
        st, nw = w.write_batch(data, offs[s:e + 1])
        if st:
            return ["rg %d: oracle write failed (%d at %d)" % (r, st, nw)]
        w.close()
        want = chunk_table(w.file_bytes())
        del w
        if want[0][0] != cnt:
            return ["rg %d (records %d..): GPU cut after %d records, oracle after %d" % (r, s, cnt, want[0][0])]
        bad = []
        for c, ((gb, gm), (ob, om)) in enumerate(zip(got[r][1], want[0][1])):
            if gm != om:
                bad.append("rg %d col %s: column metadata differs" % (r, schema.columns[c][0]))
            if gb != ob:
                i = next((j for j in range(min(len(gb), len(ob))) if gb[j] != ob[j]), min(len(gb), len(ob)))
                bad.append("rg %d col %s: chunk bytes differ at %d (len %d vs %d)" % (r, schema.columns[c][0], i,
                                                                                     len(gb), len(ob)))
        return bad

    with ThreadPoolExecutor(_workers()) as ex:   # ctypes releases the GIL inside the oracle
        for b in ex.map(one, range(len(got))):
            errs += b
    return errs


