"""Minimal Parquet file walker for tests: Thrift-compact reader + page listing.

Used to (a) decompress every page with pyarrow's Snappy (independent decoder),
(b) diff two files page by page when a byte-parity test fails.
"""
import struct


class TReader:
    def __init__(self, buf, pos=0):
        self.b = buf
        self.p = pos

    def byte(self):
        v = self.b[self.p]
        self.p += 1
        return v

    def varint(self):
        r = s = 0
        while True:
            c = self.byte()
            r |= (c & 0x7F) << s
            s += 7
            if not c & 0x80:
                return r

    def zz(self):
        v = self.varint()
        return (v >> 1) ^ -(v & 1)

    def read_value(self, t):
        if t in (1, 2):
            return t == 1
        if t == 3:
            return self.byte()
        if t in (4, 5, 6):
            return self.zz()
        if t == 7:
            v = struct.unpack_from("<d", self.b, self.p)[0]
            self.p += 8
            return v
        if t == 8:
            n = self.varint()
            v = bytes(self.b[self.p:self.p + n])
            self.p += n
            return v
        if t in (9, 10):
            h = self.byte()
            n = h >> 4
            et = h & 15
            if n == 15:
                n = self.varint()
            return [self.read_value(et) for _ in range(n)]
        if t == 12:
            return self.read_struct()
        raise ValueError("thrift type %d" % t)

    def read_struct(self):
        out = {}
        last = 0
        while True:
            h = self.byte()
            if h == 0:
                return out
            t = h & 15
            d = h >> 4
            fid = last + d if d else self.zz()
            last = fid
            out[fid] = self.read_value(t)


def footer(buf):
    assert buf[:4] == b"PAR1" and buf[-4:] == b"PAR1"
    n = struct.unpack_from("<I", buf, len(buf) - 8)[0]
    start = len(buf) - 8 - n
    return TReader(buf, start).read_struct()


def pages(buf):
    """Yield dicts: rg, col, offset, header(dict), body(bytes) for every page of every chunk."""
    fm = footer(buf)
    for rgi, rg in enumerate(fm[4]):
        for ci, cc in enumerate(rg[1]):
            md = cc[3]
            pos = md[9]
            end = pos + md[7]
            while pos < end:
                r = TReader(buf, pos)
                h = r.read_struct()
                body = bytes(buf[r.p:r.p + h[3]])
                yield {"rg": rgi, "col": ci, "offset": pos, "header": h, "body": body}
                pos = r.p + h[3]


def decompress_pages(buf, codec_name="snappy"):
    import pyarrow as pa
    out = []
    for pg in pages(buf):
        h = pg["header"]
        # DataPageV2 (type 3): rl + dl bytes stay uncompressed in front of the values
        lv = (h[8][5] + h[8][6]) if h[1] == 3 else 0
        if codec_name == "snappy" and h[2] == lv:
            raw = pg["body"]
        elif codec_name == "snappy":
            raw = pg["body"][:lv] + pa.decompress(pg["body"][lv:], decompressed_size=h[2] - lv, codec="snappy",
                                                  asbytes=True)
        elif codec_name == "gzip":   # one gzip member per page (Python's gzip module: header, CRC, ISIZE checked)
            import gzip
            raw = pg["body"][:lv] + gzip.decompress(pg["body"][lv:])
        else:
            raw = pg["body"]
        assert len(raw) == h[2]
        out.append((pg, raw))
    return out


def first_difference(a, b):
    """Human-readable first page-level difference between two files (or None)."""
    if a == b:
        return None
    pa_ = list(pages(a)) if a[-4:] == b"PAR1" else []
    pb_ = list(pages(b)) if b[-4:] == b"PAR1" else []
    for x, y in zip(pa_, pb_):
        if x["header"] != y["header"] or x["body"] != y["body"]:
            i = next((k for k in range(min(len(x["body"]), len(y["body"]))) if x["body"][k] != y["body"][k]), None)
            return ("rg %d col %d page@%d: header %r vs %r; body len %d vs %d; first diff byte %r" %
                    (x["rg"], x["col"], x["offset"], x["header"], y["header"], len(x["body"]), len(y["body"]), i))
    if len(pa_) != len(pb_):
        return "page count %d vs %d" % (len(pa_), len(pb_))
    i = next((k for k in range(min(len(a), len(b))) if a[k] != b[k]), None)
    return "pages equal; file bytes differ at %r (len %d vs %d) — footer" % (i, len(a), len(b))
