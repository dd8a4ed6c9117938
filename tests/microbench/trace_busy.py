"""GPU busy profile of a rocprofv3 kernel trace (test-side analysis, no GPU needed):
  python tests/microbench/trace_busy.py <run_kernel_trace.csv> [bucket_ms]
Prints the span, the union of kernel intervals (busy time: some kernel in flight), the mean
number of kernels in flight while busy, per-kernel totals, and a per-bucket busy fraction
timeline (where in a step the chip idles).  Kernel durations include time a dispatched
kernel waits for CUs, so "busy" means "some dispatch outstanding", not "CUs full"."""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    bucket = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    t0, t1 = rows[0][0], max(e for _, e, _ in rows)
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    tot = sum(e - s for s, e, _ in rows)
    print("span %.1f ms, busy %.1f ms (%.1f %%), kernel time %.1f ms, mean in flight while busy %.2f, %d dispatches"
          % ((t1 - t0) / 1e6, busy / 1e6, 100.0 * busy / (t1 - t0), tot / 1e6, tot / max(1, busy), len(rows)))
    per = collections.defaultdict(lambda: [0, 0])
    for s, e, k in rows:
        per[k][0] += 1
        per[k][1] += e - s
    print("%-40s %8s %10s %8s" % ("kernel", "calls", "total ms", "avg us"))
    for k, (c, d) in sorted(per.items(), key=lambda kv: -kv[1][1])[:25]:
        print("%-40s %8d %10.2f %8.1f" % (k[:40], c, d / 1e6, d / c / 1e3))
    # busy fraction per bucket
    nb = int((t1 - t0) / (bucket * 1e6)) + 1
    cov = [0.0] * nb
    merged = []
    for s, e, _ in rows:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    for s, e in merged:
        a, b = (s - t0) / 1e6, (e - t0) / 1e6
        while a < b:
            k = int(a // bucket)
            nxt = min(b, (k + 1) * bucket)
            cov[k] += nxt - a
            a = nxt
    print("busy fraction per %.0f ms bucket:" % bucket)
    print(" ".join("%3d" % int(100 * c / bucket) for c in cov))


if __name__ == "__main__":
    main()
