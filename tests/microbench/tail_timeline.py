"""Test infrastructure: a writer step's tail from a rocprofv3 kernel + memory-copy trace (csv):
steps split at gaps in the H2D stream; per step the last H2D, the job starts (k_decode) near
the end with their record counts, and when the last kernel and the last D2H end.
  python tests/microbench/tail_timeline.py <trace dir> [gap_ms]"""
import csv
import glob
import sys

d = sys.argv[1]
gap = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
K = list(csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])))
M = list(csv.DictReader(open(glob.glob(d + "/*memory_copy_trace.csv")[0])))
for r in K + M:
    r["s"] = int(r["Start_Timestamp"])
    r["e"] = int(r["End_Timestamp"])
h2d = sorted((m for m in M if m["Direction"].endswith("HOST_TO_DEVICE")), key=lambda m: m["s"])
d2h = sorted((m for m in M if m["Direction"].endswith("DEVICE_TO_HOST")), key=lambda m: m["s"])
groups = [[h2d[0]]]
for a, b in zip(h2d, h2d[1:]):
    if b["s"] - a["e"] > gap * 1e6:
        groups.append([])
    groups[-1].append(b)
dec = sorted((r for r in K if "k_decode" in r["Kernel_Name"]), key=lambda r: r["s"])
for i, g in enumerate(groups):
    s0 = g[0]["s"]
    s1 = groups[i + 1][0]["s"] if i + 1 < len(groups) else 1 << 62
    last_h = max(m["e"] for m in g)
    kk = [r for r in K if s0 <= r["s"] < s1]
    dd = [r for r in dec if s0 <= r["s"] < s1]
    oo = [m for m in d2h if s0 <= m["s"] < s1]
    if not kk:
        continue
    last_k = max(r["e"] for r in kk)
    last_o = max((m["e"] for m in oo), default=0)
    print("step %d: %d H2D, last H2D end %.1f ms, last kernel end %.1f, last D2H end %.1f, jobs %d"
          % (i, len(g), (last_h - s0) / 1e6, (last_k - s0) / 1e6, (last_o - s0) / 1e6, len(dd)))
    for r in dd:
        if r["s"] > last_h - 40e6:
            # the job's kernels: same queue, from its decode to the next decode on that queue
            nxt = [x["s"] for x in dd if x["Queue_Id"] == r["Queue_Id"] and x["s"] > r["s"]]
            end = min(nxt) if nxt else s1
            jk = [x for x in kk if x["Queue_Id"] == r["Queue_Id"] and r["s"] <= x["s"] < end]
            print("   job decode at %7.1f  records %8d  q%s  its kernels end %7.1f  kernel time %.1f ms"
                  % ((r["s"] - s0) / 1e6, int(r["Grid_Size_X"]), r["Queue_Id"], (max(x["e"] for x in jk) - s0) / 1e6,
                     sum(x["e"] - x["s"] for x in jk) / 1e6))
