"""Test infrastructure: summarise a rocprofv3 CSV trace (kernel + memory-copy + HIP API) of a
writer run: which HIP calls produce the blit kernels (__amd_rocclr_copyBuffer / fillBuffer),
their sizes (grid), durations, and whether they ran while k_snappy_seg held the CUs.
  python tests/microbench/trace_copies.py TRACE_DIR > summary.txt"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]


def rows(pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fp:
            out += list(csv.DictReader(fp))
    return out


K = rows("*kernel_trace.csv")
A = rows("*hip_api_trace.csv")
M = rows("*memory_copy_trace.csv")
print("kernel rows", len(K), "api rows", len(A), "memcpy rows", len(M))
if K:
    print("kernel cols", list(K[0].keys()))
if A:
    print("api cols", list(A[0].keys()))
if M:
    print("memcpy cols", list(M[0].keys()))
api = {r["Correlation_Id"]: r for r in A}
segs = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in K if "k_snappy_seg" in r["Kernel_Name"])


def in_seg(t0, t1):
    for a, b in segs:
        if a < t1 and t0 < b:
            return True
    return False


agg = collections.defaultdict(lambda: [0, 0.0, 0, 0])
for r in K:
    n = r["Kernel_Name"]
    if "rocclr" not in n:
        continue
    a = api.get(r["Correlation_Id"], {})
    fn = a.get("Function", "?")
    t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    grid = int(r.get("Grid_Size_X", r.get("Grid_Size", "0")) or 0)
    gb = "grid<=1k" if grid <= 1024 else "grid<=64k" if grid <= 65536 else "grid>64k"
    key = (n.split("(")[0][:40], fn, a.get("Thread_Id", "?"), gb)
    e = agg[key]
    e[0] += 1
    e[1] += (t1 - t0) / 1e6
    e[2] += 1 if in_seg(t0, t1) else 0
    e[3] = max(e[3], grid)
print("\nblit kernels: (kernel, HIP call, host thread, grid bucket) -> calls, total ms, calls overlapping k_snappy_seg, max grid")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%-42s %-26s tid %-8s %-10s %5d %9.3f ms  seg-overlap %5d  maxgrid %d" % (k[0], k[1], k[2], k[3], v[0], v[1], v[2], v[3]))
magg = collections.defaultdict(lambda: [0, 0.0, 0])
for r in M:
    a = api.get(r["Correlation_Id"], {})
    key = (r.get("Direction", "?"), a.get("Function", "?"))
    e = magg[key]
    e[0] += 1
    e[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    e[2] += int(r.get("Size", r.get("Bytes", "0")) or 0)
print("\nSDMA copies: (direction, HIP call) -> calls, total ms, bytes")
for k, v in sorted(magg.items(), key=lambda kv: -kv[1][1]):
    print("%-30s %-26s %5d %9.3f ms %14d B" % (k[0], k[1], v[0], v[1], v[2]))
fc = collections.Counter(r["Function"] for r in A)
print("\nHIP calls:", ", ".join("%s %d" % kv for kv in fc.most_common(25)))
