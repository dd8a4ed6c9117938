"""Test infrastructure: full-size writer file vs the oracle row group by row group, with a
per-page diagnosis of any mismatching chunk (is the page content different, or only its Snappy
bytes?).  python tests/microbench/diag_fullsize.py KIND SEED N CODEC [REPS]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("", "tests", "synth", "kafka-parquet-writer_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402

import gpu_helpers  # noqa: E402
import kpw  # noqa: E402
import oracle  # noqa: E402
import pqwalk  # noqa: E402
import synth  # noqa: E402

MiB = 1024 * 1024
kind, seed, n, codec = int(sys.argv[1]), int(sys.argv[2], 0), int(sys.argv[3]), int(sys.argv[4])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 1
schema = synth.SCHEMAS[kind]
data, offs = synth.generate(kind, seed, n)
props = oracle.make_props(block_size=128 * MiB, page_size=128 * MiB, codec=codec, enable_dictionary=True)


def pages_of_chunk(fb, rg, col):
    return [pg for pg in pqwalk.pages(fb) if pg["rg"] == rg and pg["col"] == col]


def raw(pg):
    h = pg["header"]
    if codec == 0 or h[2] == h[3] and pg["body"] == b"":
        return pg["body"]
    return pa.decompress(pg["body"], decompressed_size=h[2], codec="snappy", asbytes=True)


for rep in range(reps):
    pf = kpw.ParquetFile(None, kpw.Schema(schema.message_name, schema.columns, schema.proto_class),
                         kpw.ParquetProperties(compression_codec_name=codec))
    for a in range(0, n, 500_000):
        b = min(n, a + 500_000)
        pf.write_batch((data[int(offs[a]):int(offs[b])], (offs[a:b + 1] - offs[a]).astype(np.uint64)))
    pf.close()
    fb = pf.file_bytes()
    del pf
    errs = gpu_helpers.check_row_groups(schema, data, offs, fb, props)
    print("rep %d codec %d: %d mismatches %s" % (rep, codec, len(errs), errs[:6]), flush=True)
    seen = set()
    starts = np.cumsum([0] + [rg[3] for rg in pqwalk.footer(fb)[4]])
    for e in errs:
        w = e.split()
        r, cname = int(w[1]), w[3].rstrip(":")
        c = [x[0] for x in schema.columns].index(cname)
        if (r, c) in seen:
            continue
        seen.add((r, c))
        s, cnt = int(starts[r]), int(starts[r + 1] - starts[r])
        ow = oracle.OracleWriter(schema, props)
        ow.write_batch(data, offs[s:min(n, s + cnt + gpu_helpers.AHEAD) + 1])
        ow.close()
        ofb = ow.file_bytes()
        gp, op = pages_of_chunk(fb, r, c), pages_of_chunk(ofb, 0, c)
        print("  rg %d col %s: pages gpu %d oracle %d" % (r, cname, len(gp), len(op)))
        for k, (g, o) in enumerate(zip(gp, op)):
            if g["header"] == o["header"] and g["body"] == o["body"]:
                continue
            gr, orr = raw(g), raw(o)
            same = gr == orr
            i = next((j for j in range(min(len(gr), len(orr))) if gr[j] != orr[j]), min(len(gr), len(orr)))
            print("    page %d type %d: header gpu %r oracle %r; uncompressed content %s (first diff %d of %d/%d)" % (
                k, g["header"][1], {x: g["header"][x] for x in (2, 3)}, {x: o["header"][x] for x in (2, 3)},
                "IDENTICAL" if same else "DIFFERENT", i, len(gr), len(orr)))
            if same and codec == 1:   # locate the differing Snappy fragment(s)
                gb, ob = g["body"], o["body"]
                j = next((q for q in range(min(len(gb), len(ob))) if gb[q] != ob[q]), None)
                print("      compressed bodies first differ at byte %r (of %d / %d)" % (j, len(gb), len(ob)))
                if os.environ.get("DIAG_DUMP"):
                    import struct
                    with open(os.environ["DIAG_DUMP"], "wb") as f:
                        f.write(struct.pack("<Q", len(orr)))
                        f.write(orr)
                    print("      page dumped to %s" % os.environ["DIAG_DUMP"])
            elif not same:
                print("      gpu %s\n      orc %s" % (gr[max(0, i - 32):i + 32].hex(), orr[max(0, i - 32):i + 32].hex()))
    sys.stdout.flush()
