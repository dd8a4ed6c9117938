"""Summarise one workload's rocprofv3 output (gpurun_out/prof_<tag>_<workload>/) into committed files:
  profiles/<tag>_<workload>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_<workload>_pmc_traffic.json   per-kernel FETCH_SIZE / WRITE_SIZE per launch, bytes
  profiles/<tag>_<workload>_summary.md         kernel table + traffic + the bench line

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB.  MI355X_MICROARCH.md (HBM section):
on gfx950 FETCH_SIZE reports exactly half the bytes of a WIDE COALESCED STREAMING read
(16 B per lane); other access widths are uncalibrated.  So the x2 correction is applied only
to the kernels listed in STREAMING_16B (their reads are 16 B/lane streams); every other
kernel's fetch is reported raw (random probes, byte/8-byte loads, scalar loads).  Ratios
between variants of one kernel are unaffected either way.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# kernels whose HBM reads are 16-byte-per-lane coalesced streams (the calibrated case)
STREAMING_16B = {"kpw::k_snappy_s_rest"}   # emit_literal_wide: 16 B/lane streaming copies of incompressible input


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def counters(path, counter):
    d = collections.defaultdict(list)
    if not os.path.exists(path):
        return d
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            d[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return d


def main(tag, workload):
    src = os.path.join(ROOT, "gpurun_out", "prof_%s_%s" % (tag, workload))
    dst = os.path.join(ROOT, "profiles")
    name = "%s_%s" % (tag, workload)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, name + "_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    fetch = counters(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counters(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    traffic = {}
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(k, [0])) / max(1, len(fetch.get(k, [])))
        w = sum(write.get(k, [0])) / max(1, len(write.get(k, [])))
        corr = 2.0 if k in STREAMING_16B else 1.0
        traffic[k] = {"fetch_bytes_raw": round(f), "fetch_correction": corr, "fetch_bytes": round(corr * f),
                      "write_bytes": round(w), "traffic_bytes": round(corr * f + w), "launches": len(fetch.get(k, []))}
    json.dump({"tag": tag, "workload": workload, "unit": "bytes per launch", "streaming_16b_x2": sorted(STREAMING_16B),
               "kernels": traffic}, open(os.path.join(dst, name + "_pmc_traffic.json"), "w"), indent=1)
    bench = ""
    log = os.path.join(src, "trace.log")
    if os.path.exists(log):
        lines = [l for l in open(log) if l.startswith("{")]
        bench = lines[-1].strip() if lines else ""
    with open(os.path.join(dst, name + "_summary.md"), "w") as fo:
        fo.write("# Profile %s — bench.py --workload %s, rocprofv3\n\n" % (tag, workload))
        fo.write("Commands: `profiles/profile_round.sh %s %s` (trace pass: bench --steps 3 --warmup 1; PMC passes: "
                 "--steps 2 --warmup 1; every pass also runs the resident-encode leg).  FETCH is raw except for "
                 "the 16 B/lane streaming kernels %s (x2, MI355X_MICROARCH.md HBM section).\n\n"
                 % (tag, workload, sorted(STREAMING_16B)))
        fo.write("Counter GB/s = (FETCH + WRITE bytes per launch) / average launch time, i.e. the HBM traffic a "
                 "kernel actually moves, against the 8.0 TB/s HBM peak (MI355X_MICROARCH.md); the algorithmic "
                 "roofline of the dominant kernel (K7) is in the bench line's `roofline` object.\n\n")
        fo.write("| kernel | calls | total ms | avg ms | % | FETCH GB/launch | WRITE GB/launch | counter GB/s | of 8 TB/s |\n")
        fo.write("|---|---|---|---|---|---|---|---|---|\n")
        for r in rows[:40]:
            k = short(r["Name"])
            t = traffic.get(k, {})
            avg_ms = float(r["AverageNs"]) / 1e6
            rate = (t["traffic_bytes"] / (avg_ms * 1e-3) / 1e9) if t and avg_ms > 0 else None
            fo.write("| `%s` | %s | %.3f | %.3f | %s | %s | %s | %s | %s |\n" % (
                k, r["Calls"], float(r["TotalDurationNs"]) / 1e6, avg_ms, r["Percentage"][:5],
                "%.3f" % (t["fetch_bytes"] / 1e9) if t else "-", "%.3f" % (t["write_bytes"] / 1e9) if t else "-",
                "%.0f" % rate if rate is not None else "-", "%.1f %%" % (rate / 80.0) if rate is not None else "-"))
        if bench:
            fo.write("\nBench line of the trace pass (profiler attached):\n\n```\n%s\n```\n" % bench)
    print("wrote profiles/%s_{kernel_stats.csv,pmc_traffic.json,summary.md}" % name)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "c2")
