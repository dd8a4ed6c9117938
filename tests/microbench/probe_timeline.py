"""Test infrastructure: per-probe timeline of a per-record loop's rocprofv3 database (kernels
view): probes split at each k_decode; span, GPU-busy and the largest gaps inside a probe
(host syncs / launch latency), and the host time between probes.
  python tests/microbench/probe_timeline.py results.db"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end from kernels order by start").fetchall()
probes, cur = [], []
for r in rows:
    if r[0].startswith("kpw::k_decode") and cur:
        probes.append(cur)
        cur = []
    cur.append(r)
if cur:
    probes.append(cur)
probes = [p for p in probes if any(k[0].startswith("kpw::k_decode") for k in p)]
n = len(probes)
span = sum(p[-1][2] - p[0][1] for p in probes) / n / 1e3
busy = sum(sum(k[2] - k[1] for k in p) for p in probes) / n / 1e3
between = [probes[i + 1][0][1] - probes[i][-1][2] for i in range(n - 1)]
between.sort()
print("probes %d  span %.1f us  busy %.1f us  kernels/probe %.1f" % (n, span, busy, sum(len(p) for p in probes) / n))
print("between probes: median %.1f us  mean %.1f us" % (between[len(between) // 2] / 1e3, sum(between) / len(between) / 1e3))
gaps = collections.defaultdict(list)
for p in probes:
    for a, b in zip(p, p[1:]):
        g = b[1] - a[2]
        if g > 0:
            gaps[(a[0].split("(")[0][:40], b[0].split("(")[0][:40])].append(g)
tot = sorted(((sum(v) / n / 1e3, k, len(v)) for k, v in gaps.items()), reverse=True)
print("largest inside-probe gaps (us per probe, after -> before, count):")
for t, k, m in tot[:15]:
    print("  %7.1f  %s -> %s  (%d)" % (t, k[0], k[1], m))
kt = collections.defaultdict(float)
for p in probes:
    for k in p:
        kt[k[0].split("(")[0][:50]] += (k[2] - k[1])
print("kernel time per probe (us):")
for name, t in sorted(kt.items(), key=lambda x: -x[1])[:15]:
    print("  %7.1f  %s" % (t / n / 1e3, name))
