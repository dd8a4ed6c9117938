"""Helpers for the GPU parity tests: run the HIP encoder on device-resident batches and
compare, page by page, with the CPU oracle's file for the same records and properties."""
import io

import numpy as np

import oracle
import pqwalk

MiB = 1024 * 1024


def to_device(data, offsets):
    import torch
    d = torch.from_numpy(np.ascontiguousarray(data) if len(data) else np.zeros(1, np.uint8)).to("cuda")
    o = torch.from_numpy(offsets.astype(np.int64)).to("cuda")
    return d, o


def gpu_encoder_pages(schema, data, offsets, codec=0, block_size=128 * MiB, page_size=128 * MiB, dictionary=True,
                      writer_version=1, enc=None):
    """Returns (row_groups, [(rg, col, [page dicts with 'body'])]) from the HIP encoder
    (a fresh one, or `enc` to reuse an encoder across batches)."""
    import kpw
    import torch
    if enc is None:
        enc = kpw.Encoder(kpw.Schema(schema.message_name, schema.columns, schema.proto_class), codec=codec,
                          block_size=block_size, page_size=page_size, enable_dictionary=dictionary,
                          writer_version=writer_version)
    d, o = to_device(data, offsets)
    torch.cuda.synchronize()
    info = enc.encode(d.data_ptr(), o.data_ptr(), len(offsets) - 1, final=True)
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
                             writer_version=kw.get("writer_version", 1))


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
