#!/usr/bin/env python
"""bench.py — Parquet encode throughput on MI355X (BASELINE.json metric, config C2).

Workload: Rec8 records (proto2, ~62 B), 100 M per GPU, dictionary on,
SNAPPY, 128 MiB row groups, 128 MiB pages (reference default).  One "step" = one pass of
the flush path over the whole device-resident batch: K1 decode -> row-group planner ->
K2 dictionary / K3 RLE / K4 PLAIN / K6 stats -> K7 Snappy, every page of every row group
produced in HBM (kpw_encoder_encode, final=1).  Record bytes are resident in HBM before
timing starts; page bytes stay in HBM (the PCIe-inclusive rate is reported separately).

value = sum over ranks of serialized record-value bytes / max-over-ranks wall time (GB/s,
the reference's `written.bytes` definition, KafkaProtoParquetWriter.java:115,280).
Multi-GPU: one process per GPU, each encoding its own partition (weak scaling, no
data-path collective).  The barrier/max use torch.distributed (RCCL).
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in ("kafka-parquet-writer_amd", "synth"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402

MiB = 1024 * 1024
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)


def log(msg):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench] " + msg, file=sys.stderr, flush=True)


# SURVEY.md §8(d) configurations that fit one GPU: kind, records per GPU, seed, description.
# C2 is the headline (BASELINE.json metric); C3 / C4 are extra measurement lines.
WORKLOADS = {
    "c2": (1, 100_000_000, 0xC0FFEE02, "C2: Rec8 (8 cols)"),
    "c3": (3, 10_000_000, 0xC0FFEE03, "C3: Wide telemetry (ts + 199 optional cols, 30% null)"),
    "c4": (2, 20_000_000, 0xC0FFEE04, "C4: HighCard (ts, uuid, JSON blob, code)"),
}


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


def cpu_baseline(kind, seed, sample_records, threads):
    """The CPU oracle (a C restatement of parquet-mr 1.10.1's write path, kind "port") on a
    bounded sample of the same workload: `threads` independent files (one per thread, like
    the reference's threadCount writers), each encoding sample_records/threads records."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    import synth
    per = max(1, sample_records // threads)
    chunks = [synth.generate(kind, seed, per, start=i * per) for i in range(threads)]
    props = oracle.make_props(codec=oracle.SNAPPY)
    total_bytes = sum(int(o[-1]) for _, o in chunks)
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
    return dict(value=round(total_bytes / dt / 1e9, 4), unit="GB/s", cores=threads, kind="port",
                sample="%d %s records (%d per thread, %.1f MB), SNAPPY, 128 MiB row groups, %d threads, %.2f s"
                       % (per * threads, synth.SCHEMAS[kind].message_name.split(".")[-1], per, total_bytes / 1e6, threads, dt),
                records_per_s=round(per * threads / dt, 1))


# K7 as launched by launch_snappy (k_snappy.hip): the register-table kernel on every fragment,
# then the batched LDS kernel on the fragments it gave up on; timed together (one HIP-event
# pair on the encoder's stream) and reported as one kernel step
SNAPPY_KERNELS = ("kpw::k_snappy_v", "kpw::k_snappy_s_rest")
SNAPPY_NAME = "K7 kpw::k_snappy_v + kpw::k_snappy_s_rest"


def pmc_traffic(kernels):
    """HBM bytes per launch summed over `kernels` from the newest profiles/<tag>_pmc_traffic.json
    (separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, gfx950 x2 FETCH correction;
    profiles/summarize.py).  Returns (bytes, source file) or (None, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    ks = [d.get("kernels", {}).get(k) for k in kernels]
    if not all(ks):
        return None, None
    return int(sum(k["traffic_bytes"] for k in ks)), os.path.relpath(files[-1], ROOT)


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


def timed_steps(step, steps, warmup, dist=None, sync=lambda: None):
    """W untimed warmup steps, then exactly K timed steps bracketed by barrier + device sync
    on both sides; returns (max-over-ranks elapsed seconds, per-step results)."""
    for _ in range(warmup):
        step()
    sync()
    if dist:
        dist.barrier()
    sync()
    out = []
    t0 = time.perf_counter()
    for _ in range(steps):
        out.append(step())
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2",
                    help="SURVEY §8(d) configuration (c2 = the BASELINE.json metric's workload)")
    ap.add_argument("--records", type=int, default=0, help="records per GPU (default: the workload's, C2: 100 M)")
    ap.add_argument("--codec", type=int, default=1, help="0 UNCOMPRESSED, 1 SNAPPY (C2)")
    ap.add_argument("--cpu-sample", type=int, default=24_000_000,
                    help="records for the CPU baseline sample (~1.5 GB, ~16 s of single-core oracle work)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    torch.cuda.set_device(local_rank)
    dist = dist_init(world, local_rank)

    import kpw
    import synth
    kind, default_records, wseed, wdesc = WORKLOADS[args.workload]
    schema = synth.SCHEMAS[kind]
    args.records = args.records or default_records
    seed = (wseed if world == 1 else 0xC0FFEE05 + rank) if args.workload == "c2" else wseed + 0x100 * rank
    t0 = time.perf_counter()
    data, offs = synth.generate(kind, seed, args.records)
    log("generated %d records (%.2f GB) in %.1fs" % (args.records, len(data) / 1e9, time.perf_counter() - t0))
    d_data = torch.from_numpy(data).to("cuda")
    d_off = torch.from_numpy(offs.view(np.int64)).to("cuda")
    nbytes = int(offs[-1])
    n = args.records
    del data
    enc = kpw.Encoder(kpw.Schema(schema.message_name, schema.columns, schema.proto_class),
                      device=local_rank, codec=args.codec, block_size=128 * MiB, page_size=128 * MiB)
    torch.cuda.synchronize()

    def step():
        return enc.encode(d_data.data_ptr(), d_off.data_ptr(), n, final=True)

    stage_acc = np.zeros(10)

    def timed():
        info = step()
        stage_acc[:] += np.array(enc.stage_times(), dtype=np.float64)[:10]
        return info

    for _ in range(args.warmup):
        step()
    elapsed, infos = timed_steps(timed, args.steps, 0, dist, torch.cuda.synchronize)
    info = infos[-1]
    # whole-job units: every rank's own partition
    total_bytes = reduce_scalar(nbytes * args.steps, dist)
    total_records = reduce_scalar(n * args.steps, dist)

    # per-step page statistics (for algorithmic bytes of the compression kernel)
    pages = enc.pages()
    unc = sum(p["uncompressed_size"] for p in pages)
    comp = sum(p["compressed_size"] for p in pages)
    stages = (stage_acc / args.steps).tolist()
    nrg = info.num_row_groups

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    ms_per_step = elapsed / args.steps * 1e3
    value = total_bytes / elapsed / 1e9
    rec_s = total_records / elapsed
    # K1 decode: algorithmic bytes = record bytes + offsets in; columnar values out
    # (ts 8, user_id 4, status 4, price 8, score 8, key16 8+4, region 8+4 per record,
    #  presence/boolean bits n/8 per optional column + flag bits, raw sizes 4 per record)
    k1_bytes = nbytes + 8 * (n + 1) + decode_out_bytes(schema, n)
    names = ["decode", "plan", "stats+dict", "rle", "layout+plain+write", "compress", "metadata", "total",
             "k_decode", "k_snappy"]
    stage = dict(zip(names, [round(x, 3) for x in stages]))
    k_dec_ms = stages[8] if len(stages) > 8 else stages[0]
    k_sn_ms = stages[9] if len(stages) > 9 else stages[5]
    # the two kernels timed live with HIP events on the encoder's stream (kpw_encoder_stage_times
    # [8], [9]); K7 = one launch of the Snappy fragment kernel over all pages of the batch
    kern = {"kpw::k_decode": (k1_bytes, k_dec_ms, ("kpw::k_decode",)),
            SNAPPY_NAME: (unc + comp, k_sn_ms, SNAPPY_KERNELS)}
    dom = max(kern, key=lambda k: kern[k][1])
    ab, ams, knames = kern[dom]
    achieved = ab / (ams * 1e-3) / 1e9 if ams > 0 else 0.0
    traffic, tsrc = pmc_traffic(knames)
    roof = dict(bound="hbm", kernel=dom, achieved=round(achieved, 2), peak=HBM_PEAK_GBPS, unit="GB/s",
                frac=round(achieved / HBM_PEAK_GBPS, 5),
                traffic=(round(traffic / (ams * 1e-3) / 1e9, 2) if traffic else None),
                traffic_bytes_per_launch=traffic, traffic_source=tsrc, algorithmic_bytes_per_launch=int(ab),
                avg_launch_ms=round(ams, 4))
    cpu = None
    if not args.no_cpu_baseline and world == 1:   # rank 0 at N=1 only
        threads = args.cpu_threads or min(16, os.cpu_count() or 8)
        sample = args.cpu_sample
        if args.workload != "c2":   # the same ~1.5 GB of wire bytes as the C2 sample
            sample = max(threads, int(sample * 62 / max(1.0, nbytes / n)))
        cpu = cpu_baseline(kind, seed, sample, threads)
    out = {
        "metric": "Parquet encode GB/s + records/sec (whole node) at 1/2/4/8 MI355X vs CPU writer",
        "value": round(value, 4), "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic (counter-based proto2 %s generator; no broker, in-memory record source)"
                               % schema.message_name.split(".")[-1],
        "config": {"workload": "%s, %d records/GPU, PLAIN_DICTIONARY + %s, 128 MiB row groups, "
                               "128 MiB pages, parquet-mr 1.10.1 v1 semantics"
                               % (wdesc, n, "SNAPPY" if args.codec else "UNCOMPRESSED"),
                   "records_per_gpu": n, "bytes_per_gpu": nbytes, "row_groups_per_gpu": nrg,
                   "codec": "SNAPPY" if args.codec else "UNCOMPRESSED", "parallelism": "partition-sharded x%d" % world},
        "records_per_s": round(rec_s, 1),
        "stage_ms": stage,
        "pages": {"uncompressed_bytes": int(unc), "compressed_bytes": int(comp), "count": len(pages)},
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
