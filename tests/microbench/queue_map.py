"""Stream -> hardware queue map of a rocprofv3 kernel trace (test-side analysis): for every
Stream_Id the Queue_Ids its dispatches went to, and per queue the streams sharing it.
  python tests/microbench/queue_map.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

sq = collections.defaultdict(collections.Counter)
for r in csv.DictReader(open(sys.argv[1])):
    sq[int(r["Stream_Id"])][int(r["Queue_Id"])] += 1
qs = collections.defaultdict(list)
for st, c in sorted(sq.items()):
    q = c.most_common(1)[0][0]
    qs[q].append(st)
    print("stream %4d -> queues %s" % (st, dict(c)))
print("queues:", {q: v for q, v in sorted(qs.items())})
