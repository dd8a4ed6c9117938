"""Summarise one workload's rocprofv3 output (gpurun_out/prof_<tag>_<workload>/) into committed files:
  profiles/<tag>_<workload>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_<workload>_pmc_traffic.json   per-kernel FETCH_SIZE / WRITE_SIZE, per encode JOB
  profiles/<tag>_<workload>_summary.md         per-kernel table, K7 reconciliation, stage rooflines

Every pass runs `bench.py --no-resident`, so every kernel launch belongs to a writer encode job
and a job is exactly one `kpw::k_decode` launch.  Counters and times are therefore normalised
PER JOB (= per launch of the dominant kernel group, the unit of the bench line's `roofline`):
a kernel launched twice per job (k_snappy_v, k_snappy_s_rest) counts twice.

  pmc_traffic.py  `python profiles/summarize.py pmc <tag> <workload>`  (after the two PMC passes)
  full summary    `python profiles/summarize.py all <tag> <workload>`  (after the trace pass)

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB.  MI355X_MICROARCH.md (HBM section):
on gfx950 FETCH_SIZE reports exactly half the bytes of a WIDE COALESCED STREAMING read
(16 B per lane); other access widths are uncalibrated.  So the x2 correction is applied only
to the kernels listed in STREAMING_16B (their reads are 16 B/lane streams); every other
kernel's fetch is reported raw (random probes, byte/8-byte loads, scalar loads).
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HBM_PEAK = 8.0e12   # B/s, MI355X_MICROARCH.md

# kernels whose HBM reads are 16-byte-per-lane coalesced streams (the calibrated case)
STREAMING_16B = {
    "kpw::k_decode",         # record bytes staged into LDS with 16 B/lane coalesced loads (k_decode.hip)
    "kpw::k_snappy_s_rest",  # emit_literal_wide: 16 B/lane streaming copies of incompressible input
}
JOB_KERNEL = "kpw::k_decode"   # one launch per encode job
# the K7 HIP-event window of the bench line (engine.cpp: kev_[2] .. kev_[3])
K7 = ["kpw::k_snappy_v", "kpw::k_snappy_s_rest", "kpw::k_snappy_seg", "kpw::k_snappy_page_sizes", "kpw::k_snappy_copy"]


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def counters(path, counter):
    """kernel -> list of per-dispatch byte counts"""
    d = collections.defaultdict(list)
    if not os.path.exists(path):
        return d
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            d[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return d


def pmc(tag, workload):
    src = os.path.join(ROOT, "gpurun_out", "prof_%s_%s" % (tag, workload))
    fetch = counters(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counters(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    jf, jw = len(fetch.get(JOB_KERNEL, [])), len(write.get(JOB_KERNEL, []))
    if not jf or not jw:
        raise SystemExit("no %s dispatches in the PMC passes" % JOB_KERNEL)
    traffic = {}
    for k in sorted(set(fetch) | set(write)):
        corr = 2.0 if k in STREAMING_16B else 1.0
        f_raw = sum(fetch.get(k, [])) / jf
        w = sum(write.get(k, [])) / jw
        traffic[k] = {"calls_per_job": round(len(fetch.get(k, [])) / jf, 3), "fetch_bytes_raw_per_job": round(f_raw),
                      "fetch_correction": corr, "fetch_bytes_per_job": round(corr * f_raw),
                      "write_bytes_per_job": round(w), "traffic_bytes_per_job": round(corr * f_raw + w)}
    # traffic relative to the algorithmic bytes of the same jobs: every pass runs --warmup 0, so
    # its bench line's launches are exactly the pass's jobs (eager jobs vary in size with timing)
    ratio = None
    bf = bench_line(os.path.join(src, "fetch.log"))
    bw = bench_line(os.path.join(src, "write.log"))
    if bf and bw and bf.get("roofline") and bw.get("roofline"):
        af = bf["roofline"]["algorithmic_bytes_per_launch"] * bf["roofline"]["launches"]
        aw = bw["roofline"]["algorithmic_bytes_per_launch"] * bw["roofline"]["launches"]
        if bf["roofline"]["launches"] == jf and bw["roofline"]["launches"] == jw and af > 0 and aw > 0:
            kf = sum((2.0 if k in STREAMING_16B else 1.0) * sum(fetch.get(k, [])) for k in K7)
            kw = sum(sum(write.get(k, [])) for k in K7)
            ratio = round(kf / af + kw / aw, 4)
    out = {"tag": tag, "workload": workload, "unit": "bytes per encode job (= per launch of the bench line's "
           "dominant kernel group); every dispatch of a kernel in the pass summed, divided by the pass's %s "
           "dispatches" % JOB_KERNEL, "jobs": {"fetch_pass": jf, "write_pass": jw},
           "streaming_16b_x2": sorted(STREAMING_16B), "k7_kernels": K7,
           "k7_traffic_bytes_per_job": sum(traffic[k]["traffic_bytes_per_job"] for k in K7 if k in traffic),
           "k7_traffic_over_algorithmic": ratio,
           "k7_ratio_note": "K7 FETCH (x2 on 16 B/lane streams) / K7 algorithmic bytes of the fetch pass + K7 WRITE / "
                            "K7 algorithmic bytes of the write pass (algorithmic = page bytes in + compressed bytes out, "
                            "from each pass's bench line; launches == jobs)",
           "kernels": traffic}
    path = os.path.join(ROOT, "profiles", "%s_%s_pmc_traffic.json" % (tag, workload))
    json.dump(out, open(path, "w"), indent=1)
    print("wrote", os.path.relpath(path, ROOT))
    return out


def bench_line(path):
    if not os.path.exists(path):
        return None
    lines = [l for l in open(path) if l.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def full(tag, workload):
    src = os.path.join(ROOT, "gpurun_out", "prof_%s_%s" % (tag, workload))
    dst = os.path.join(ROOT, "profiles")
    name = "%s_%s" % (tag, workload)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, name + "_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    jobs_t = next(int(r["Calls"]) for r in rows if short(r["Name"]) == JOB_KERNEL)
    pm = json.load(open(os.path.join(dst, name + "_pmc_traffic.json")))
    tr = pm["kernels"]
    bl = bench_line(os.path.join(src, "trace.log"))
    with open(os.path.join(dst, name + "_summary.md"), "w") as fo:
        fo.write("# Profile %s — bench.py --workload %s --no-resident, rocprofv3\n\n" % (tag, workload))
        fo.write("Commands: `profiles/profile_round.sh %s %s`: two PMC passes (FETCH_SIZE, WRITE_SIZE; bench --steps 3 "
                 "--warmup 0) then the kernel-trace pass (bench --steps 3 --warmup 0), all `--no-resident "
                 "--no-cpu-baseline`, so every launch is a writer encode job.  Jobs: trace pass %d, fetch pass %d, "
                 "write pass %d (`%s` dispatches).  Per-job figures = every dispatch of the kernel in the pass / the "
                 "pass's jobs.  FETCH is raw except for the 16 B/lane streaming kernels %s (x2, MI355X_MICROARCH.md "
                 "HBM section).\n\n" % (tag, workload, jobs_t, pm["jobs"]["fetch_pass"], pm["jobs"]["write_pass"],
                                        JOB_KERNEL, sorted(STREAMING_16B)))
        fo.write("| kernel | calls/job | ms/job | avg ms/call | % | FETCH MB/job | WRITE MB/job | counter GB/s |\n")
        fo.write("|---|---|---|---|---|---|---|---|\n")
        for r in rows[:45]:
            k = short(r["Name"])
            t = tr.get(k)
            ms_job = float(r["TotalDurationNs"]) / 1e6 / jobs_t
            rate = t["traffic_bytes_per_job"] / (ms_job * 1e-3) / 1e9 if t and ms_job > 0 else None
            fo.write("| `%s` | %.2f | %.3f | %.3f | %s | %s | %s | %s |\n" % (
                k, int(r["Calls"]) / jobs_t, ms_job, float(r["AverageNs"]) / 1e6, r["Percentage"][:5],
                "%.1f" % (t["fetch_bytes_per_job"] / 1e6) if t else "-", "%.1f" % (t["write_bytes_per_job"] / 1e6) if t else "-",
                "%.0f" % rate if rate is not None else "-"))
        # K7 reconciliation: trace-pass kernel time per job vs the bench line's HIP-event window
        k7_ms = sum(float(r["TotalDurationNs"]) for r in rows if short(r["Name"]) in K7) / 1e6 / jobs_t
        k7_tr = pm["k7_traffic_bytes_per_job"]
        fo.write("\n## K7 (dominant kernel group) per job\n\n")
        fo.write("- kernels: %s\n" % ", ".join("`%s` x%.2f" % (k, tr[k]["calls_per_job"]) for k in K7 if k in tr))
        fo.write("- kernel time per job (trace pass, sum of the K7 kernels' durations / jobs): **%.3f ms**\n" % k7_ms)
        fo.write("- counter traffic per job (FETCH + WRITE, call-weighted): **%.1f MB**\n" % (k7_tr / 1e6))
        if bl and bl.get("roofline"):
            ro = bl["roofline"]
            ab = ro["algorithmic_bytes_per_launch"]
            fo.write("- bench line (same trace pass): HIP-event K7 window %.3f ms per launch over %d launches; "
                     "algorithmic bytes per launch %d (page bytes in + compressed bytes out)\n"
                     % (ro["avg_launch_ms"], ro["launches"], ab))
            fo.write("- achieved = %d B / %.3f ms = **%.1f GB/s**, frac = %.1f / 8000 = **%.5f**\n"
                     % (ab, ro["avg_launch_ms"], ab / (ro["avg_launch_ms"] * 1e-3) / 1e9,
                        ab / (ro["avg_launch_ms"] * 1e-3) / 1e9, ab / (ro["avg_launch_ms"] * 1e-3) / HBM_PEAK))
            if pm.get("k7_traffic_over_algorithmic"):
                rr = pm["k7_traffic_over_algorithmic"]
                fo.write("- counter traffic / algorithmic bytes (PMC passes, same jobs: %s) = **%.2fx**; for this pass's "
                         "launches: %.2f x %d B = **%.1f MB per launch** (the bench line's `traffic`)\n"
                         % (pm.get("k7_ratio_note", ""), rr, rr, ab, rr * ab / 1e6))
            else:
                fo.write("- counter traffic / algorithmic bytes = %.1f MB / %.1f MB = **%.2fx**\n"
                         % (k7_tr / 1e6, ab / 1e6, k7_tr / max(1, ab)))
            st = bl.get("stage_roofline")
            if st:
                fo.write("\n## Encode stages per job (HIP events on the encoder stream, algorithmic bytes of "
                         "SURVEY §8d)\n\n| stage | kernels | device ms/job | algorithmic MB/job | GB/s | of 8 TB/s |\n"
                         "|---|---|---|---|---|---|\n")
                for k, v in st.items():
                    fo.write("| %s | %s | %.3f | %.1f | %.0f | %.2f %% |\n" % (
                        k, v.get("kernels", ""), v["ms_per_job"], v["alg_bytes_per_job"] / 1e6, v["gbps"], 100 * v["frac"]))
            fo.write("\nBench line of the trace pass (profiler attached):\n\n```\n%s\n```\n" % json.dumps(bl))
    print("wrote profiles/%s_{kernel_stats.csv,summary.md}" % name)


if __name__ == "__main__":
    mode, tag = sys.argv[1], sys.argv[2]
    wl = sys.argv[3] if len(sys.argv) > 3 else "c2"
    if mode == "pmc":
        pmc(tag, wl)
    else:
        full(tag, wl)
