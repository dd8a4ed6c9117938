"""PCIe-inclusive rate of the ParquetFile drop-in (kpw_writer_* C-ABI).

bench.py times the encoder with the batch already resident in HBM (the `value` the driver
records).  This script times the whole boundary the reference's caller sees
(KafkaProtoParquetWriter.WorkerThread: write per record KPW:277, close KPW:326-337): record
bytes start in host memory, go through kpw_writer_write in poll()-sized batches, and the file
(footer included) ends in host memory.  H2D of the wire bytes, the encode, D2H of the pages
and the host file assembly are all inside the timed region.  It is never bench.py's `value`.

  python bench_writer.py [--records 100000000] [--batch 500000] [--steps 2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in ("kafka-parquet-writer_amd", "synth"):
    sys.path.insert(0, os.path.join(ROOT, p))

MiB = 1024 * 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=100_000_000)
    ap.add_argument("--batch", type=int, default=500_000, help="records per write call (a poll() batch)")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--codec", type=int, default=1)
    args = ap.parse_args()

    import kpw
    import synth
    data, offs = synth.generate(synth.KIND_REC8, 0xC0FFEE02, args.records)
    nbytes = int(offs[-1])
    schema = kpw.Schema(synth.REC8.message_name, synth.REC8.columns, synth.REC8.proto_class)
    props = kpw.ParquetProperties(block_size=128 * MiB, compression_codec_name=args.codec, page_size=128 * MiB)
    dptr = data.ctypes.data

    def one_file():
        t0 = time.perf_counter()
        f = kpw.ParquetFile(None, schema, props)
        L = f._L
        t1 = time.perf_counter()
        for i in range(0, args.records, args.batch):
            j = min(args.records, i + args.batch)
            f._check(L.kpw_writer_write(f._h, dptr, offs[i:].ctypes.data, j - i), "write")
        t2 = time.perf_counter()
        f.close()
        dt = time.perf_counter() - t0
        if os.environ.get("KPW_TRACE") == "1":
            print("[bench_writer] open %.1f ms, writes %.1f ms, close %.1f ms" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3,
                  (time.perf_counter() - t2) * 1e3), file=sys.stderr, flush=True)
        size = len(f.file_bytes())
        return dt, size

    one_file()  # warm-up (device buffers, code objects)
    times = []
    size = 0
    for _ in range(args.steps):
        dt, size = one_file()
        times.append(dt)
    best = min(times)
    med = float(np.median(times))
    print(json.dumps({
        "metric": "ParquetFile writer path GB/s (host record bytes in -> file bytes out, PCIe-inclusive)",
        "value": round(nbytes / med / 1e9, 4), "best": round(nbytes / best / 1e9, 4), "unit": "GB/s",
        "records_per_s": round(args.records / med, 1), "seconds": [round(t, 3) for t in times],
        "records": args.records, "wire_bytes": nbytes, "file_bytes": size, "batch_records": args.batch,
        "config": "C2 Rec8, SNAPPY, 128 MiB row groups, one file, in-memory output"}), flush=True)


if __name__ == "__main__":
    main()
