"""Summarise one round's rocprofv3 output (gpurun_out/prof_<tag>/) into committed files:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc_traffic.json   per-kernel FETCH_SIZE/WRITE_SIZE per launch, in bytes
  profiles/<tag>_summary.md         per-step kernel table + traffic + the bench line
FETCH_SIZE/WRITE_SIZE are reported by rocprofv3 in KiB.  On gfx950 FETCH_SIZE counts half
the bytes of wide coalesced streaming reads (MI355X_MICROARCH.md, HBM section): the json
keeps the raw value and a x2-corrected one; `traffic` in bench.py uses the corrected
fetch + write.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    dst = os.path.join(ROOT, "profiles")
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, tag + "_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    fetch = counters(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counters(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    traffic = {}
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(k, [0])) / max(1, len(fetch.get(k, [])))
        w = sum(write.get(k, [0])) / max(1, len(write.get(k, [])))
        traffic[k] = {"fetch_bytes_raw": round(f), "fetch_bytes_x2": round(2 * f), "write_bytes": round(w),
                      "traffic_bytes": round(2 * f + w), "launches": len(fetch.get(k, []))}
    json.dump({"tag": tag, "unit": "bytes per launch", "kernels": traffic},
              open(os.path.join(dst, tag + "_pmc_traffic.json"), "w"), indent=1)
    bench = ""
    log = os.path.join(src, "trace.log")
    if os.path.exists(log):
        lines = [l for l in open(log) if l.startswith("{")]
        bench = lines[-1].strip() if lines else ""
    steps = 4  # warmup 1 + steps 3 in the trace pass
    with open(os.path.join(dst, tag + "_summary.md"), "w") as fo:
        fo.write("# Profile %s — C2 bench (100 M Rec8, SNAPPY, 128 MiB row groups), rocprofv3\n\n" % tag)
        fo.write("Commands: `profiles/profile_round.sh %s` (trace pass: bench --steps 3 = 4 encodes incl. warmup;"
                 " PMC passes: bench --steps 2).\n\n" % tag)
        fo.write("| kernel | calls | total ms | avg ms | ms / encode | % | FETCH x2 GB/launch | WRITE GB/launch |\n")
        fo.write("|---|---|---|---|---|---|---|---|\n")
        for r in rows[:30]:
            k = short(r["Name"])
            t = traffic.get(k, {})
            fo.write("| `%s` | %s | %.3f | %.3f | %.3f | %s | %s | %s |\n" % (
                k, r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e6,
                float(r["TotalDurationNs"]) / 1e6 / steps, r["Percentage"][:5],
                "%.3f" % (t["fetch_bytes_x2"] / 1e9) if t else "-", "%.3f" % (t["write_bytes"] / 1e9) if t else "-"))
        if bench:
            fo.write("\nBench line of the trace pass (profiler attached):\n\n```\n%s\n```\n" % bench)
    print("wrote profiles/%s_{kernel_stats.csv,pmc_traffic.json,summary.md}" % tag)


if __name__ == "__main__":
    main(sys.argv[1])
