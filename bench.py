#!/usr/bin/env python
"""bench.py — Parquet encode throughput on MI355X, the BASELINE.json metric as defined.

Metric (BASELINE.md:16-19): serialized record-value bytes consumed (the
reference's `written.bytes` meter, KafkaProtoParquetWriter.java:115,280) divided by the wall
time from the first ParquetFile write until the last file is closed.  A step is one complete
file per writer through the ParquetFile drop-in (kpw_writer_*, writer.cpp): record batches
start in host memory (pinned, where polled Kafka batches land: north_star), are written in
poll()-sized batches (500 k records), cross PCIe, are encoded (K1..K7), come back as pages and
are assembled into an in-memory file (headers, footer).  H2D, encode, D2H and file assembly
are all inside the timed region.

Workloads (--workload):
  c2  Rec8, 100 M records/GPU, PLAIN_DICTIONARY + SNAPPY, 128 MiB row groups (BASELINE metric)
  c3  Wide telemetry (ts + 199 optional cols, 30% null), 10 M records/GPU
  c4  HighCard (ts, uuid, JSON blob, code), 20 M records/GPU
  c5  64-partition topic: 8 partitions per GPU, one writer per partition on its own thread,
      125 M records/GPU (15.625 M per partition, seed 0xC0FFEE05 + partition)
Timed steps cycle over two distinct record batches (different seeds) for c2-c4; every step
opens fresh writers, so nothing an encoder learns (K7's longest-first fragment order) carries
between steps.

Secondary keys: `resident_encode` (kpw_encoder_encode on a batch already in HBM, the r01
headline), `c4` (the C4 writer line, 2 steps), `bulk_multipage` (C2 bulk writes with 1 MiB
pages inside 128 MiB row groups, 2 steps), `c5` (BASELINE config 5 at its shape: 8 concurrent
writers of 15.625 M Rec8 records each, 2 steps), `gzip` (the C2 writer line with
CompressionCodecName.GZIP, 2 steps), `per_record` / `per_record_multipage` /
`per_record_64k` (the reference's write + getDataSize loop at 128 MiB / 1 MiB / 64 KiB pages, the
oracle's same loops in `cpu_baseline`), `roofline` (the dominant kernel, timed with HIP events on the encoder's stream inside
the timed writer steps; algorithmic bytes per launch), `roofline.pipeline_frac` (sum of
algorithmic bytes over sum of device time of every encode stage, §8d), a measured device copy
ceiling, and `cpu_baseline` (the CPU oracle — a C restatement of parquet-mr 1.10.1 — doing the
same work: host records in -> files out, one file per thread, median of 5 runs).

Multi-GPU: one process per GPU (torchrun), each writing its own partitions (weak scaling, no
data-path collective).  The barrier/max use torch.distributed (RCCL).

Every rank binds itself to the CPUs of its GPU's NUMA node before allocating anything (pinned
batches, writer threads next to the card's PCIe root; KPW_BENCH_NO_NUMA=1 skips it).  Measured on
one box, 3 runs each: 27.5 / 28.3 / 30.0 GB/s bound, 26.2 / 26.8 / 23.3 unbound.
"""
import argparse
import ctypes
import glob
import json
import os
import sys
import threading
import time

# Hardware queues per process (HIP's default is 4): eight writers' stream sets (four streams
# each) share fewer queues; 8 measured C5 31.7 -> 33.8 GB/s (3 paired runs, r05aw), C2 / C4
# unchanged.  The deployment setting DESIGN.md recommends; an explicit value is kept.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in ("kafka-parquet-writer_amd", "synth"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402

MiB = 1024 * 1024
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)
POLL_BATCH = 500_000    # records per write call (a poll() batch)
# kernels inside the K7 HIP-event window (engine.cpp kev_[2]..kev_[3]); profiles/summarize.py K7
K7_KERNELS = ["k_snappy_v x2", "k_snappy_s_rest x2", "k_snappy_seg", "k_snappy_page_sizes", "k_snappy_copy"]
# what each HIP-event stage of kpw_encoder_stage_times covers (engine.cpp ev_[0..6])
STAGE_KERNELS = {
    "decode": "K1 k_decode",
    "plan": "prefix scans (k_mj_*), def-level RLE structure (k_rle_*, k_phase_*, k_r_*), events, K8 k_plan",
    "stats_dict": "K6 k_chunk_stats, k_str_minmax; K2 k_dict_insert, k_dict_firsts, k_dict_ids",
    "rle": "K3 structure of the level / id streams (k_rle_*, k_phase_*, k_r_*)",
    "layout_plain_write": "layout; K4 k_plain, k_plain_bool, k_dict_page; K3 k_rle_write_*",
    "compress": "K7 window + page size D2H and the host's longest-first fragment order",
}


def log(msg):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench] " + msg, file=sys.stderr, flush=True)


# kind, records per GPU, seed, description
WORKLOADS = {
    "c2": (1, 100_000_000, 0xC0FFEE02, "C2: Rec8 (8 cols), SNAPPY, 128 MiB row groups"),
    "c3": (3, 10_000_000, 0xC0FFEE03, "C3: Wide telemetry (ts + 199 optional cols, 30% null), SNAPPY"),
    "c4": (2, 20_000_000, 0xC0FFEE04, "C4: HighCard (ts, uuid, JSON blob, code), SNAPPY"),
    "c5": (1, 125_000_000, 0xC0FFEE05, "C5: Rec8, 8 partitions per GPU, one writer per partition, SNAPPY"),
}
C5_PARTS_PER_GPU = 8


def partition_seeds(workload, rank, world):
    """Record sets of one rank: a list (timed steps cycle over it) of lists of partition seeds
    (one writer per partition).  Ranks never share a partition (weak scaling, no exchange)."""
    kind, _, wseed, _ = WORKLOADS[workload]
    if workload == "c5":   # 64-partition topic: partitions rank*8 .. rank*8+7
        return [[wseed + rank * C5_PARTS_PER_GPU + p for p in range(C5_PARTS_PER_GPU)]]
    if workload == "c2":
        seed = wseed if world == 1 else 0xC0FFEE05 + rank * C5_PARTS_PER_GPU
    else:
        seed = wseed + 0x100 * rank
    return [[seed + 0x1000 * k] for k in range(2)]   # two distinct batches


def decode_out_bytes(schema, n):
    """K1 algorithmic output bytes: 8 B per 64-bit value, 4 B per 32-bit value, 12 B (offset +
    length) per string, 1 bit per bool, 1 bit of presence per optional column, 4 B raw size."""
    import synth
    per = 4
    bits = 0
    for _, _, t, label in schema.columns:
        if t == synth.BOOL:
            bits += 1
        elif t in (synth.STRING, synth.BYTES):
            per += 12
        elif t in (synth.INT64, synth.UINT64, synth.DOUBLE, synth.FIXED64, synth.SFIXED64, synth.SINT64):
            per += 8
        else:
            per += 4
        if label == synth.OPTIONAL:
            bits += 1
    return n * per + (bits * n) // 8


def column_bytes(schema, n, record_bytes):
    """Columnar value bytes the chunk kernels read once (fixed-width values, string offset +
    length + the string bytes themselves, bits): the K2/K4/K6 input."""
    return decode_out_bytes(schema, n) - 4 * n + max(0, record_bytes - 2 * n * len(schema.columns)) // 2


def stage_bytes(schema, st):
    """Algorithmic (compulsory) bytes per encode stage, SURVEY §8d, from a writer's totals.
    Keys follow kpw_encoder_stage_times: decode, plan, stats+dict, rle, layout+plain+write,
    compress."""
    n, rb = st["records"], st["record_bytes"]
    unc, comp = st["page_bytes_uncompressed"], st["page_bytes_compressed"]
    cols = column_bytes(schema, n, rb)
    nopt = sum(1 for c in schema.columns if c[3] == 1)
    return {
        "decode": rb + 8 * n + decode_out_bytes(schema, n),                 # K1: wire in, columns out
        "plan": 4 * n + 8 * n + nopt * n // 8,                              # raw sizes in, prefix out, presence bits
        "stats_dict": 2 * cols + 4 * n,                                     # K6 + K2: columns in (twice), ids out
        "rle": 4 * n + nopt * n // 8 + 0,                                   # K3: ids / levels in (packed out counted in layout)
        "layout_plain_write": cols + unc,                                   # K4: values in, page bodies out
        "compress": unc + comp,                                             # K7: pages in, compressed out
    }


def pmc_traffic(workload):
    """K7 HBM bytes per encode job from the newest profiles/*_<workload>_pmc_traffic.json: separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `bench.py --no-resident` (every launch a
    writer job), each K7 kernel's dispatches summed and divided by the pass's jobs (calls per job
    weighted), the gfx950 x2 FETCH correction on 16 B/lane streaming kernels only
    (profiles/summarize.py).  Returns (bytes, file) or (None, None)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_%s_pmc_traffic.json" % workload)))
    for f in reversed(files):
        d = json.load(open(f))
        if d.get("k7_traffic_over_algorithmic"):   # r03c on: traffic relative to the same jobs' bytes
            return ("ratio", float(d["k7_traffic_over_algorithmic"])), os.path.relpath(f, ROOT)
        if "k7_traffic_bytes_per_job" in d:   # per-job format (r03a/b)
            return ("bytes", int(d["k7_traffic_bytes_per_job"])), os.path.relpath(f, ROOT)
    return None, None


def dist_init(world, local_rank, backend="nccl"):
    """One process per GPU (torchrun env). backend "nccl" is RCCL on ROCm; tests use gloo."""
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist
    if backend == "nccl":
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend=backend)
    return dist


def timed_steps(step, steps, warmup, dist=None, sync=lambda: None, on_start=None):
    """W untimed warmup steps, then exactly K timed steps bracketed by barrier + device sync
    on both sides; returns (max-over-ranks elapsed seconds, per-step results).  on_start runs
    (untimed) right before the timed region."""
    for i in range(warmup):
        step(i)
    sync()
    if dist:
        dist.barrier()
    sync()
    if on_start:
        on_start()
    out = []
    t0 = time.perf_counter()
    for i in range(steps):
        out.append(step(warmup + i))
    sync()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    return reduce_scalar(elapsed, dist, "max"), out


def reduce_scalar(x, dist=None, op="sum"):
    """Scalar all-reduce across ranks (bookkeeping only; the data path has no collective)."""
    if not dist:
        return x
    import torch
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def rank_memory(dist=None, pinned_sets=()):
    """This rank's host-memory budget (N ranks share a node's host memory): the
    library's pinned-cache cap (48 GB / LOCAL_WORLD_SIZE unless KPW_PIN_CACHE_GB is set,
    memcache.cpp), its live and idle pinned bytes, the record sets this rank pinned, and the
    worst case (sets + live + cap) maxed over ranks.  Reads allocator counters only (no GPU call)."""
    import kpw
    from kpw import _lib
    st = _lib.cache_stats()
    sets = sum(int(d.nbytes) + int(o.nbytes) for d, o in pinned_sets)
    budget = sets + st["pin_cache_cap"] + max(0.0, st["pin_live"] - sets)
    return dict(local_world_size=int(os.environ.get("LOCAL_WORLD_SIZE", "1")),
                pin_cache_cap_gb=round(st["pin_cache_cap"] / 1e9, 3), dev_cache_cap_gb=round(st["dev_cache_cap"] / 1e9, 3),
                record_sets_pinned_gb=round(sets / 1e9, 3), pinned_live_gb=round(st["pin_live"] / 1e9, 3),
                pinned_idle_gb=round(st["pin_idle"] / 1e9, 3),
                pinned_budget_gb_max_over_ranks=round(reduce_scalar(budget, dist, "max") / 1e9, 3))


def write_file(kpw, schema, props, data, offs, device, batch=POLL_BATCH):
    """One ParquetFile through the drop-in: batches straight from (pinned) host memory.
    Returns (file size, pipeline stats); the stats carry the host wall of the writer's phases
    (open, writes, close, stats, free: `phase_*_ms`), so the line shows where a step went."""
    t0 = time.perf_counter()
    pf = kpw.ParquetFile(None, schema, props, device=device)
    L, h = pf._L, pf._h
    base = data.ctypes.data
    optr = offs.ctypes.data
    n = len(offs) - 1
    t1 = time.perf_counter()
    # kpw_writer_write_async: each poll batch's DMA is queued behind the previous one (the
    # batches are never modified, so the "until the next call returns" reuse rule holds)
    for a in range(0, n, batch):
        b = min(n, a + batch)
        st = L.kpw_writer_write_async(h, base, optr + 8 * a, b - a)   # absolute offsets into `data`
        if st:
            pf._check(st, "write")
    t2 = time.perf_counter()
    pf.close()
    t3 = time.perf_counter()
    size, stats = L.kpw_writer_data_size(h), pf.pipeline_stats()   # after close: the file's length
    t4 = time.perf_counter()
    pf.__del__()   # the writer (and its in-memory file) is released inside the step
    t5 = time.perf_counter()
    stats.update(phase_open_ms=(t1 - t0) * 1e3, phase_writes_ms=(t2 - t1) * 1e3, phase_close_ms=(t3 - t2) * 1e3,
                 phase_stats_ms=(t4 - t3) * 1e3, phase_free_ms=(t5 - t4) * 1e3)
    if os.environ.get("KPW_TRACE") == "1":
        print("[bench] writer: open %.1f ms, writes %.1f ms, close %.1f ms, stats %.1f ms, free %.1f ms" % (
            (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3, (t5 - t4) * 1e3),
            file=sys.stderr, flush=True)
    return size, stats


PHASES = ("open", "writes", "close", "stats", "free")


def cache_delta(before, after):
    """Allocator calls and their host ms between two kpw_cache_stats snapshots."""
    keys = ("dev_malloc_n", "dev_malloc_ms", "dev_free_n", "dev_free_ms", "pin_malloc_n", "pin_malloc_ms", "pin_free_n",
            "pin_free_ms", "dev_retry", "dev_sync_n", "dev_sync_ms", "gate_admits", "gate_wait_ms")
    return {k: round(after.get(k, 0.0) - before.get(k, 0.0), 2) for k in keys}


def copy_ceiling(device, nbytes=2 << 30):
    """Measured device-to-device copy rate (read + write bytes / time), the practical HBM roof."""
    import torch
    src = torch.empty(nbytes, dtype=torch.uint8, device="cuda:%d" % device)
    dst = torch.empty_like(src)
    dst.copy_(src)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    del src, dst
    torch.cuda.empty_cache()
    return round(2 * nbytes / (ms * 1e-3) / 1e9, 1)


def cpu_baseline(kind, seed, sample_records, threads, runs=5):
    """The CPU oracle (C restatement of parquet-mr 1.10.1's write path, kind "port") doing the
    same work as a writer step: host record bytes in -> a closed in-memory file out, one file
    per thread (the reference's threadCount writers).  1 warm-up + `runs` timed runs, median."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    import synth
    per = max(1, sample_records // threads)
    chunks = [synth.generate(kind, seed, per, start=i * per) for i in range(threads)]
    props = oracle.make_props(codec=oracle.SNAPPY)
    total_bytes = sum(int(o[-1]) for _, o in chunks)
    times = []
    for r in range(runs + 1):
        errs = []

        def work(i):
            try:
                d, o = chunks[i]
                oracle.encode_file(synth.SCHEMAS[kind], d, o, props)
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        ts = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        dt = time.perf_counter() - t0
        if errs:
            raise errs[0]
        if r:
            times.append(dt)
    med = float(np.median(times))
    return dict(value=round(total_bytes / med / 1e9, 4), unit="GB/s", cores=threads, kind="port",
                sample="%d %s records (%d per thread, %.1f MB), SNAPPY, 128 MiB row groups, one in-memory file per "
                       "thread, %d threads, median of %d runs (%s s)"
                       % (per * threads, synth.SCHEMAS[kind].message_name.split(".")[-1], per, total_bytes / 1e6,
                          threads, runs, ", ".join("%.2f" % t for t in times)),
                records_per_s=round(per * threads / med, 1))


def per_record_leg(kpw, schema, sschema, kind, seed, n, device, max_file_size, page_size, runs=3):
    """The reference's unchanged WorkerThread loop (KafkaProtoParquetWriter.java:268-285,306-308):
    ONE kpw_writer_write + ONE kpw_writer_data_size per record through the C-ABI (the two
    downcalls a JVM host makes, driven from C: synth/loop.c), rotating files when getDataSize()
    >= maxFileSize, on a C2-shaped stream in ordinary (unpinned) host memory (a JVM byte[]).
    The CPU oracle's same loop is timed in the cpu_baseline leg (cpu_baseline_per_record)."""
    import synth
    data, offs = synth.generate(kind, seed + 0x77, n)
    nbytes = int(offs[-1])
    L = kpw.load_library()
    props = kpw.ParquetProperties(block_size=128 * MiB, compression_codec_name=kpw.SNAPPY, page_size=page_size)
    pf = kpw.ParquetFile(None, schema, props, device=device)   # warm-up: library caches, first encode
    synth.per_record_loop("kpw", L.kpw_writer_write, L.kpw_writer_data_size, pf._h, data, offs, 0, min(n, 20000),
                          max_file_size)
    pf.close()
    pf.__del__()
    walls = []
    for _ in range(runs):   # the loop over all n records, `runs` times: the median is reported
        t0 = time.perf_counter()
        done = files = 0
        while done < n:
            pf = kpw.ParquetFile(None, schema, props, device=device)
            got, full, st, _ = synth.per_record_loop("kpw", L.kpw_writer_write, L.kpw_writer_data_size, pf._h, data, offs,
                                                     done, n - done, max_file_size)
            if st:
                pf._check(st, "per-record write")
            pf.close()
            pf.__del__()
            files += 1
            done += got
        walls.append(time.perf_counter() - t0)
    dt = float(np.median(walls))
    return dict(records=n, bytes=nbytes, records_per_s=round(n / dt, 1), gbps=round(nbytes / dt / 1e9, 4),
                wall_s=round(dt, 3), runs_wall_s=[round(w, 3) for w in walls], statistic="median of %d runs" % runs,
                files=files, max_file_size=max_file_size, page_size=page_size,
                calls_per_record="1 kpw_writer_write (n=1) + 1 kpw_writer_data_size, from C (synth/loop.c)",
                reference_sizing_hint_records_per_s=300000)


def writer_leg(kpw, kind, seed, n, device, steps, warmup, page_size=128 * MiB, sets=None, codec=None):
    """Secondary writer-path line (same drop-in and timing as the headline, fewer steps): another
    workload (C4) or another page size (pageSize(...) < blockSize, KafkaProtoParquetWriter.java:656-659
    -> ParquetFile.java:47: bulk writes with page cuts inside row groups)."""
    import synth
    sschema = synth.SCHEMAS[kind]
    schema = kpw.Schema(sschema.message_name, sschema.columns, sschema.proto_class)
    if sets is None:
        sets = [synth.generate(kind, seed + 0x1000 * k, n, alloc=kpw.pinned_empty) for k in range(2)]
    codec = kpw.SNAPPY if codec is None else codec
    props = kpw.ParquetProperties(block_size=128 * MiB, compression_codec_name=codec, page_size=page_size)
    from kpw import _lib
    for i in range(warmup):
        write_file(kpw, schema, props, sets[i % 2][0], sets[i % 2][1], device)
    c0 = _lib.cache_stats()
    t0 = time.perf_counter()
    nb = 0
    file_bytes = 0
    step_ms, phases = [], []
    for i in range(steps):
        d, o = sets[(warmup + i) % 2]
        t = time.perf_counter()
        size, st = write_file(kpw, schema, props, d, o, device)
        step_ms.append(round((time.perf_counter() - t) * 1e3, 1))
        phases.append(st)
        nb += int(o[-1])
        file_bytes += size
    dt = time.perf_counter() - t0
    c1 = _lib.cache_stats()
    return dict(value=round(nb / dt / 1e9, 4), unit="GB/s", records_per_s=round(steps * (len(sets[0][1]) - 1) / dt, 1),
                ms_per_step=round(dt / steps * 1e3, 3), steps=steps, warmup=warmup, records_per_step=len(sets[0][1]) - 1,
                bytes_per_step=int(nb / steps), file_bytes_per_step=int(file_bytes / steps), page_size=page_size,
                step_ms=step_ms,
                writer_phase_ms_mean={ph: round(float(np.mean([st["phase_%s_ms" % ph] for st in phases])), 2) for ph in PHASES},
                h2d_gbps=round(nb / (sum(st.get("h2d_span_ms", 0.0) for st in phases) * 1e-3) / 1e9, 2)
                if all(st.get("h2d_span_ms") for st in phases) else None,
                lookback_fallbacks=int(sum(st.get("lookback_fallbacks", 0.0) for st in phases)),
                allocator_in_timed_steps=cache_delta(c0, c1),
                workload=sschema.message_name.split(".")[-1] + ", %s, 128 MiB row groups, pageSize %d"
                % ("GZIP" if codec == kpw.GZIP else "SNAPPY", page_size))


def c5_leg(kpw, device, steps, warmup):
    """Secondary writer line for BASELINE config 5 at its stated shape: the 8
    partitions of the 64-partition topic this GPU owns (seeds 0xC0FFEE05 + p), one concurrent
    kpw_writer per partition on its own thread (KafkaProtoParquetWriter.java:175-179), 125 M Rec8
    records per GPU (15.625 M per partition), SNAPPY, 128 MiB row groups, 500 k poll batches;
    one step = all 8 files closed.  Same drop-in and timing as the headline.  Reports every
    step's time, the writers' encode wall and phases, look-back fallbacks and the allocator
    calls made inside the timed steps (the in-line leg against the standalone one)."""
    import synth
    from kpw import _lib
    kind, n, wseed, wdesc = WORKLOADS["c5"]
    sschema = synth.SCHEMAS[kind]
    schema = kpw.Schema(sschema.message_name, sschema.columns, sschema.proto_class)
    props = kpw.ParquetProperties(block_size=128 * MiB, compression_codec_name=kpw.SNAPPY, page_size=128 * MiB)
    per = n // C5_PARTS_PER_GPU
    parts = [synth.generate(kind, wseed + p, per, alloc=kpw.pinned_empty) for p in range(C5_PARTS_PER_GPU)]
    nb = sum(int(o[-1]) for _, o in parts)

    def step():
        res, errs = [None] * len(parts), []

        def one(k):
            try:
                res[k] = write_file(kpw, schema, props, parts[k][0], parts[k][1], device)
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        ts = [threading.Thread(target=one, args=(k,)) for k in range(len(parts))]
        t = time.perf_counter()
        for th in ts:
            th.start()
        for th in ts:
            th.join()
        if errs:
            raise errs[0]
        return time.perf_counter() - t, res

    for _ in range(warmup):
        step()
    c0 = _lib.cache_stats()
    t0 = time.perf_counter()
    outs = [step() for _ in range(steps)]
    dt = time.perf_counter() - t0
    c1 = _lib.cache_stats()
    file_bytes = sum(size for _, res in outs for size, _ in res)
    sts = [st for _, res in outs for _, st in res]
    enc = [st.get("worker_encode_wall_ms", 0.0) for st in sts]
    return dict(value=round(nb * steps / dt / 1e9, 4), unit="GB/s", records_per_s=round(steps * per * len(parts) / dt, 1),
                ms_per_step=round(dt / steps * 1e3, 3), step_ms=[round(t * 1e3, 1) for t, _ in outs], steps=steps,
                warmup=warmup, records_per_step=per * len(parts), bytes_per_step=nb,
                file_bytes_per_step=int(file_bytes / steps), writers=len(parts), records_per_writer=per,
                writer_encode_wall_ms=dict(mean=round(float(np.mean(enc)), 2), max=round(float(np.max(enc)), 2)),
                writer_phase_ms_mean={ph: round(float(np.mean([st["phase_%s_ms" % ph] for st in sts])), 2)
                                      for ph in PHASES},
                jobs_per_writer=round(float(np.mean([st.get("jobs", 0.0) for st in sts])), 2),
                lookback_fallbacks=int(sum(st.get("lookback_fallbacks", 0.0) for st in sts)),
                allocator_in_timed_steps=cache_delta(c0, c1),
                hw_queues=os.environ.get("GPU_MAX_HW_QUEUES"),
                workload=wdesc + ", 128 MiB row groups, 500 k poll batches")


def c1_leg(kpw, device, steps=5, threads=1):
    """BASELINE config 1: 1 M Rec8 records -> ONE UNCOMPRESSED Parquet file
    (128 MiB row groups and pages), through the GPU writer (pinned host records in, closed
    in-memory file out; median of `steps` files after one warm-up) and through the CPU oracle
    (kind "port") on one core and on `threads` cores (one 1 M-record file per thread)."""
    import synth
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    kind, n, seed = synth.KIND_REC8, 1_000_000, 0xC0FFEE01
    sschema = synth.SCHEMAS[kind]
    schema = kpw.Schema(sschema.message_name, sschema.columns, sschema.proto_class)
    props = kpw.ParquetProperties(block_size=128 * MiB, compression_codec_name=kpw.UNCOMPRESSED, page_size=128 * MiB)
    data, offs = synth.generate(kind, seed, n, alloc=kpw.pinned_empty)
    nb = int(offs[-1])
    write_file(kpw, schema, props, data, offs, device)
    ts = []
    for _ in range(steps):
        t = time.perf_counter()
        write_file(kpw, schema, props, data, offs, device)
        ts.append(time.perf_counter() - t)
    gpu_s = float(np.median(ts))
    oprops = oracle.make_props(codec=oracle.UNCOMPRESSED)
    hd, ho = np.array(data), np.array(offs)
    oracle.encode_file(sschema, hd, ho, oprops)
    one = []
    for _ in range(3):
        t = time.perf_counter()
        oracle.encode_file(sschema, hd, ho, oprops)
        one.append(time.perf_counter() - t)
    one_s = float(np.median(one))

    def work():
        oracle.encode_file(sschema, hd, ho, oprops)
    th = [threading.Thread(target=work) for _ in range(threads)]
    t = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    all_s = time.perf_counter() - t
    return dict(value=round(nb / gpu_s / 1e9, 4), unit="GB/s", records_per_s=round(n / gpu_s, 1),
                ms_per_file=round(gpu_s * 1e3, 3), records=n, bytes=nb, codec="UNCOMPRESSED",
                oracle_1core=dict(value=round(nb / one_s / 1e9, 4), records_per_s=round(n / one_s, 1),
                                  ms_per_file=round(one_s * 1e3, 2), cores=1, kind="port"),
                oracle_all_cores=dict(value=round(threads * nb / all_s / 1e9, 4),
                                      records_per_s=round(threads * n / all_s, 1), cores=threads, kind="port",
                                      sample="%d files of the same 1 M records, one per thread" % threads),
                workload="C1: 1 M Rec8 records, UNCOMPRESSED, 128 MiB row groups, one file (GPU: median of %d files)"
                         % steps)


def cpu_baseline_per_record(sschema, kind, seed, n, max_file_size, page_size, runs=3):
    """CPU-baseline leg of the per-record loop: the oracle's kpwo_write + kpwo_data_size per
    record on the same records as per_record_leg, one thread (one WorkerThread)."""
    import synth
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    data, offs = synth.generate(kind, seed + 0x77, n)
    OL = oracle.lib()
    oprops = oracle.make_props(block_size=128 * MiB, page_size=page_size, codec=oracle.SNAPPY)
    walls = []
    for _ in range(runs):
        t1 = time.perf_counter()
        done = files = 0
        while done < n:
            w = oracle.OracleWriter(sschema, oprops)
            got, full, st, _ = synth.per_record_loop("oracle", OL.kpwo_write, OL.kpwo_data_size, w._h, data, offs, done,
                                                     n - done, max_file_size)
            if st:
                raise RuntimeError("oracle per-record loop status %d" % st)
            w.close()
            files += 1
            done += got
        walls.append(time.perf_counter() - t1)
    odt = float(np.median(walls))
    return dict(records=n, records_per_s=round(n / odt, 1), wall_s=round(odt, 3), runs_wall_s=[round(x, 3) for x in walls],
                statistic="median of %d runs" % runs, files=files, cores=1, kind="port")


def bind_to_gpu_numa(device):
    """One process per GPU, bound to the CPUs of the GPU's NUMA node (the usual deployment of a
    GPU worker): pinned batches, stage/page buffers and the writer's threads then sit next to the
    PCIe root of the card instead of across the socket link.  Returns the node or None."""
    import torch
    try:
        pr = torch.cuda.get_device_properties(device)
        bdf = "%04x:%02x:%02x.0" % (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id)
        node = int(open("/sys/bus/pci/devices/%s/numa_node" % bdf).read())
        if node < 0:
            return None
        cpus = set()
        for part in open("/sys/devices/system/node/node%d/cpulist" % node).read().strip().split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        cpus &= os.sched_getaffinity(0)
        if not cpus:
            return None
        os.sched_setaffinity(0, cpus)
        return node
    except (OSError, ValueError, AttributeError):
        return None


def host_threads():
    """CPU threads this process may use: the affinity mask, capped by OMP_NUM_THREADS (the GPU
    box gives one GPU's job a 16-CPU share and sets OMP_NUM_THREADS=16 accordingly)."""
    n = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(n, omp) if omp > 0 else n


def resident_encode(kpw, schema, batches, device, steps=3):
    """Secondary: kpw_encoder_encode on batches already in HBM (pages stay in HBM), cycling
    over the distinct batches; returns GB/s and the mean per-stage device ms."""
    enc = kpw.Encoder(schema, device=device, codec=1, block_size=128 * MiB, page_size=128 * MiB)
    dev = []
    for data, offs in batches:   # HBM from the library's own runtime (kpw_device_alloc)
        dev.append((kpw.DeviceBuffer.from_array(data, device), kpw.DeviceBuffer.from_array(offs, device), len(offs) - 1,
                    int(offs[-1])))
    enc.encode(dev[0][0].ptr, dev[0][1].ptr, dev[0][2], final=True)   # warm-up
    acc = np.zeros(10)
    tot_bytes = 0
    k7_bytes = 0
    t0 = time.perf_counter()
    for i in range(steps):
        d, o, n, nb = dev[(i + 1) % len(dev)]
        enc.encode(d.ptr, o.ptr, n, final=True)
        acc += np.array(enc.stage_times()[:10], dtype=np.float64)
        tot_bytes += nb
        k7_bytes += sum(p["uncompressed_size"] + p["compressed_size"] for p in enc.pages())
    dt = time.perf_counter() - t0   # kpw_encoder_encode is blocking
    for d, o, _, _ in dev:
        d.free()
        o.free()
    del dev
    names = ["decode", "plan", "stats+dict", "rle", "layout+plain+write", "compress", "metadata", "total", "k_decode",
             "k7_snappy"]
    k7_ms = acc[9] / steps
    k7_gbps = (k7_bytes / steps) / (k7_ms * 1e-3) / 1e9 if k7_ms > 0 else 0.0
    # K7 with the GPU to itself (one encoder, one launch per step): the same algorithmic bytes
    # (page bytes in + compressed bytes out) over the same HIP-event window as the main line's
    return dict(value=round(tot_bytes / dt / 1e9, 3), unit="GB/s", steps=steps,
                stage_ms=dict(zip(names, [round(x / steps, 3) for x in acc])),
                k7_roofline=dict(achieved=round(k7_gbps, 2), peak=HBM_PEAK_GBPS, unit="GB/s",
                                 frac=round(k7_gbps / HBM_PEAK_GBPS, 5),
                                 algorithmic_bytes_per_launch=int(k7_bytes / steps), avg_launch_ms=round(k7_ms, 4)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2",
                    help="SURVEY §8(d) configuration (c2 = the BASELINE.json metric's workload)")
    ap.add_argument("--records", type=int, default=0, help="records per GPU (default: the workload's)")
    ap.add_argument("--cpu-sample", type=int, default=24_000_000,
                    help="records for the CPU baseline sample (C2-equivalent bytes for other workloads)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-resident", action="store_true")
    ap.add_argument("--per-record-records", type=int, default=3_000_000,
                    help="records of the per-record leg (the reference's write + getDataSize loop; 0 = skip)")
    ap.add_argument("--per-record-max-file-mb", type=int, default=1024,
                    help="maxFileSize of the per-record leg (reference default 1 GiB, KafkaProtoParquetWriter.java:462)")
    ap.add_argument("--per-record-page-kb", type=int, default=128 * 1024,
                    help="pageSize of the per-record leg (reference default = blockSize, KafkaProtoParquetWriter.java:474)")
    ap.add_argument("--secondary-steps", type=int, default=2,
                    help="timed steps of the secondary writer legs at N=1 (c4, bulk_multipage, c5 and gzip; 0 = skip)")
    ap.add_argument("--per-record-mp-page-kb", type=int, default=1024,
                    help="pageSize of a second per-record leg with page cuts inside row groups (pageSize(...), "
                         "KafkaProtoParquetWriter.java:656-659; 0 = skip)")
    ap.add_argument("--per-record-64k-records", type=int, default=1_000_000,
                    help="records of a third per-record leg with 64 KiB pages in 128 MiB row groups, GPU and oracle "
                         "(VERDICT r4: per_record_64k; 0 = skip)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    # torch (RCCL bookkeeping, the copy-ceiling probe) bundles its own HIP runtime; it must
    # initialise before libkpw_gpu.so's, or it reports no GPU.  The data path never uses it.
    torch.cuda.set_device(local_rank)
    torch.cuda.init()
    numa = None if os.environ.get("KPW_BENCH_NO_NUMA") == "1" else bind_to_gpu_numa(local_rank)
    dist = dist_init(world, local_rank)

    import kpw
    import synth
    kind, default_records, wseed, wdesc = WORKLOADS[args.workload]
    sschema = synth.SCHEMAS[kind]
    schema = kpw.Schema(sschema.message_name, sschema.columns, sschema.proto_class)
    n = args.records or default_records
    props = kpw.ParquetProperties(block_size=128 * MiB, compression_codec_name=kpw.SNAPPY, page_size=128 * MiB)
    t0 = time.perf_counter()
    seeds = partition_seeds(args.workload, rank, world)
    per = n // len(seeds[0])
    sets = [[synth.generate(kind, sd, per, alloc=kpw.pinned_empty) for sd in ss] for ss in seeds]
    n = per * len(seeds[0])
    set_bytes = [sum(int(o[-1]) for _, o in s) for s in sets]
    log("generated %d x %d records (%.2f GB each) in pinned host memory in %.1fs"
        % (len(sets), n, set_bytes[0] / 1e9, time.perf_counter() - t0))

    step_wall = []

    def step(i):
        t = time.perf_counter()
        r = step_body(i)
        if i >= args.warmup:
            step_wall.append(time.perf_counter() - t)
        return r

    def step_body(i):
        s = sets[i % len(sets)]
        if len(s) == 1:
            size, st = write_file(kpw, schema, props, s[0][0], s[0][1], local_rank)
            return [(size, st)], set_bytes[i % len(sets)]
        res = [None] * len(s)
        errs = []

        def one(k):
            try:
                res[k] = write_file(kpw, schema, props, s[k][0], s[k][1], local_rank)
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        ts = [threading.Thread(target=one, args=(k,)) for k in range(len(s))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]
        return res, set_bytes[i % len(sets)]

    from kpw import _lib as kpw_lib
    cs = {}
    elapsed, outs = timed_steps(step, args.steps, args.warmup, dist, torch.cuda.synchronize,
                                on_start=lambda: cs.update(before=kpw_lib.cache_stats()))
    cs["after"] = kpw_lib.cache_stats()
    my_bytes = sum(b for _, b in outs)
    total_bytes = reduce_scalar(my_bytes, dist)
    total_records = reduce_scalar(n * args.steps, dist)
    # pipeline statistics of every writer of the timed steps
    agg = {}
    files = 0
    for res, _ in outs:
        for size, st in res:
            files += 1
            for k, v in st.items():
                agg[k] = agg.get(k, 0.0) + v
    file_bytes = sum(size for res, _ in outs for size, _ in res)

    # host-memory budget of the ranks sharing this node (a collective: every rank calls it)
    mem = rank_memory(dist, pinned_sets=[x for ss in sets for x in ss])

    resident = None
    if not args.no_resident and args.workload != "c5" and rank == 0:
        resident = resident_encode(kpw, schema, [s[0] for s in sets], local_rank)
    ceiling = copy_ceiling(local_rank) if rank == 0 else None

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    ms_per_step = elapsed / args.steps * 1e3
    value = total_bytes / elapsed / 1e9
    rec_s = total_records / elapsed
    jobs = max(1.0, agg.get("jobs", 1.0))
    # dominant kernel group of the timed steps: K7, timed with HIP events on the encoder's stream
    # around its kernels (engine.cpp kev_[2]..kev_[3]), one window per encode job
    k7_bytes = (agg["page_bytes_uncompressed"] + agg["page_bytes_compressed"]) / jobs
    ams = agg["k7_snappy_ms"] / jobs
    achieved = k7_bytes / (ams * 1e-3) / 1e9 if ams > 0 else 0.0
    tk, tsrc = pmc_traffic(args.workload)
    traffic, tunit = None, "HBM bytes per launch (FETCH_SIZE + WRITE_SIZE)"
    if tk and tk[0] == "ratio":   # job sizes vary (eager jobs): scale the profile's traffic/algorithmic ratio
        traffic = int(round(tk[1] * k7_bytes))
        tunit += ": the PMC passes' K7 counter bytes / K7 algorithmic bytes (%.3f, same jobs) x this line's " \
                 "algorithmic bytes per launch" % tk[1]
    elif tk:
        traffic = tk[1]
    sb = stage_bytes(sschema, agg)
    stage_ms = {"decode": agg["decode_ms"], "plan": agg["plan_ms"], "stats_dict": agg["stats_dict_ms"],
                "rle": agg["rle_ms"], "layout_plain_write": agg["layout_plain_write_ms"], "compress": agg["compress_ms"]}
    t_stages = sum(stage_ms.values())
    pipe = sum(sb.values()) / (t_stages * 1e-3) / 1e9 if t_stages > 0 else 0.0
    roof = dict(bound="hbm", kernel="K7 Snappy: " + ", ".join(K7_KERNELS), achieved=round(achieved, 2),
                peak=HBM_PEAK_GBPS, unit="GB/s", frac=round(achieved / HBM_PEAK_GBPS, 5),
                traffic=traffic, traffic_unit=tunit,
                traffic_source=tsrc, traffic_over_algorithmic=(round(traffic / k7_bytes, 3) if traffic else None),
                algorithmic_bytes_per_launch=int(k7_bytes), avg_launch_ms=round(ams, 4), launches=int(jobs),
                pipeline_achieved=round(pipe, 2), pipeline_frac=round(pipe / HBM_PEAK_GBPS, 5),
                pipeline_stage_ms=round(t_stages / jobs, 3),
                copy_ceiling=ceiling, frac_of_copy_ceiling=round(achieved / ceiling, 5) if ceiling else None)
    stage_roof = {}
    for k, ms in stage_ms.items():
        b_job, ms_job = sb[k] / jobs, ms / jobs
        g = b_job / (ms_job * 1e-3) / 1e9 if ms_job > 0 else 0.0
        stage_roof[k] = dict(kernels=STAGE_KERNELS[k], alg_bytes_per_job=int(b_job), ms_per_job=round(ms_job, 4),
                             gbps=round(g, 1), frac=round(g / HBM_PEAK_GBPS, 5))
    per_record = per_record_mp = None
    if args.per_record_records and world == 1:
        per_record = per_record_leg(kpw, schema, sschema, kind, wseed, args.per_record_records, local_rank,
                                    args.per_record_max_file_mb * MiB, args.per_record_page_kb * 1024)
        if args.per_record_mp_page_kb:   # pageSize < blockSize: page cuts inside row groups (size probes)
            per_record_mp = per_record_leg(kpw, schema, sschema, kind, wseed, args.per_record_records, local_rank,
                                           args.per_record_max_file_mb * MiB, args.per_record_mp_page_kb * 1024)
    per_record_64k = None
    if args.per_record_64k_records and world == 1:   # 64 KiB pages: a size probe every ~2-3 k records
        per_record_64k = per_record_leg(kpw, schema, sschema, kind, wseed, args.per_record_64k_records, local_rank,
                                        args.per_record_max_file_mb * MiB, 64 * 1024)
    c4_leg = bulk_mp = c5 = gz = c3_leg = c1 = None
    if args.secondary_steps and world == 1 and args.workload == "c2":
        # Secondary writer legs, in KPW_BENCH_LEGS order (a measurement knob; default below).  Each
        # starts from empty allocator caches (kpw_trim_caches: a fresh process's state) and warms
        # them in its own untimed steps; otherwise a leg inherits the previous workload's cached
        # blocks and pays hipMalloc / hipFree for its own sizes in its timed steps (r06a: C5 after
        # the C4 and multi-page legs made 229 device allocations in 3 timed steps).
        L0 = kpw.load_library()
        legs = {}

        def run_c4():   # the config where encode, not PCIe, sets the pace
            c4k, c4n, c4seed, _ = WORKLOADS["c4"]
            return writer_leg(kpw, c4k, c4seed, c4n, local_rank, args.secondary_steps, 1)

        def run_bulk():   # bulk writes with 1 MiB pages inside 128 MiB row groups
            return writer_leg(kpw, kind, wseed, n, local_rank, args.secondary_steps, 1, page_size=MiB,
                              sets=[s[0] for s in sets])

        def run_c5():   # BASELINE config 5 at its shape on this GPU
            return c5_leg(kpw, local_rank, max(3, args.secondary_steps), 2)

        def run_c3():   # BASELINE config 3 (wide telemetry schema), 10 M records, its own writer line
            c3k, c3n, c3seed, _ = WORKLOADS["c3"]
            return writer_leg(kpw, c3k, c3seed, c3n, local_rank, max(3, args.secondary_steps), 1)

        def run_gzip():   # the same C2 records with CompressionCodecName.GZIP (no BASELINE config; K7')
            return writer_leg(kpw, kind, wseed, n, local_rank, args.secondary_steps, 1, sets=[s[0] for s in sets],
                              codec=kpw.GZIP)
        runners = {"c4": run_c4, "bulk_multipage": run_bulk, "c5": run_c5, "c3": run_c3, "gzip": run_gzip}
        order = os.environ.get("KPW_BENCH_LEGS", "c5,c3,c4,bulk_multipage,gzip").split(",")
        for name in order:
            if name in runners:
                L0.kpw_trim_caches()
                legs[name] = runners[name]()
        L0.kpw_trim_caches()
        c4_leg, bulk_mp, c5, c3_leg, gz = (legs.get(k) for k in ("c4", "bulk_multipage", "c5", "c3", "gzip"))
    if args.secondary_steps and world == 1 and args.workload == "c2" and not args.no_cpu_baseline:
        c1 = c1_leg(kpw, local_rank, threads=args.cpu_threads or host_threads())   # BASELINE config 1
    cpu = None
    if not args.no_cpu_baseline and world == 1:   # rank 0 at N=1 only
        threads = args.cpu_threads or host_threads()
        sample = args.cpu_sample
        if args.workload not in ("c2", "c5"):   # the same ~1.5 GB of wire bytes as the C2 sample
            sample = max(threads, int(sample * 62 / max(1.0, set_bytes[0] / n)))
        cpu = cpu_baseline(kind, wseed, sample, threads)
        if per_record:
            cpu["per_record"] = cpu_baseline_per_record(sschema, kind, wseed, args.per_record_records,
                                                        args.per_record_max_file_mb * MiB, args.per_record_page_kb * 1024)
            per_record["oracle_records_per_s"] = cpu["per_record"]["records_per_s"]
        if per_record_mp:   # the oracle's same loop at the same page size
            cpu["per_record_multipage"] = cpu_baseline_per_record(sschema, kind, wseed, args.per_record_records,
                                                                  args.per_record_max_file_mb * MiB,
                                                                  args.per_record_mp_page_kb * 1024)
            per_record_mp["oracle_records_per_s"] = cpu["per_record_multipage"]["records_per_s"]
        if per_record_64k:
            cpu["per_record_64k"] = cpu_baseline_per_record(sschema, kind, wseed, args.per_record_64k_records,
                                                            args.per_record_max_file_mb * MiB, 64 * 1024)
            per_record_64k["oracle_records_per_s"] = cpu["per_record_64k"]["records_per_s"]
    out = {
        "metric": "Parquet encode GB/s + records/sec (whole node) at 1/2/4/8 MI355X vs CPU writer",
        "value": round(value, 4), "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (counter-based proto2 %s generator, pinned host memory; no broker: an in-memory record "
                "source in poll()-sized batches of %d)" % (sschema.message_name.split(".")[-1], POLL_BATCH),
        "config": {"workload": "%s, %d records/GPU, PLAIN_DICTIONARY + SNAPPY, 128 MiB row groups, 128 MiB pages, "
                               "parquet-mr 1.10.1 v1 semantics; ParquetFile drop-in, host bytes -> closed in-memory file "
                               "(H2D, encode, D2H, file assembly timed)" % (wdesc, n),
                   "records_per_gpu": n, "bytes_per_gpu_step": set_bytes[0], "files_per_gpu_step": len(sets[0]),
                   "codec": "SNAPPY", "parallelism": "partition-sharded x%d" % world, "numa_node": numa},
        "records_per_s": round(rec_s, 1),
        # this rank's wall per timed step (host clock around each step; the line's time is the max
        # over ranks of the whole timed region)
        "step_ms": [round(x * 1e3, 1) for x in step_wall],
        "file_bytes_per_step": int(file_bytes / max(1, args.steps)),
        "encode_jobs_per_step": round(jobs / args.steps, 2),
        "worker_encode_wall_ms_per_step": round(agg.get("worker_encode_wall_ms", 0) / args.steps, 2),
        # host wall of each writer phase (write_file), summed over the step's writers
        "writer_phase_ms_per_step": {ph: round(agg.get("phase_%s_ms" % ph, 0.0) / args.steps, 2) for ph in PHASES},
        "lookback_fallbacks": int(agg.get("lookback_fallbacks", 0)),
        # the box's PCIe as the writer saw it: record bytes / the span from the first record DMA to
        # the completion of the last (HIP timing events on the copy stream; one writer per step)
        "h2d_gbps": (round(my_bytes / (agg["h2d_span_ms"] * 1e-3) / 1e9, 2)
                     if agg.get("h2d_span_ms") and len(sets[0]) == 1 else None),
        "allocator_in_timed_steps": cache_delta(cs.get("before", {}), cs["after"]),
        "stage_ms_per_step": {k: round(v / args.steps, 3) for k, v in stage_ms.items()},
        "rank_memory": mem,
        "resident_encode": resident,
        "roofline": roof,
        "stage_roofline": stage_roof,
        "per_record": per_record,
        "per_record_multipage": per_record_mp,
        "per_record_64k": per_record_64k,
        "c4": c4_leg,
        "bulk_multipage": bulk_mp,
        "c5": c5,
        "c3": c3_leg,
        "c1": c1,
        "gzip": gz,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
