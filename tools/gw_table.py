#!/usr/bin/env python3
"""Gateway sweep table: socket_to_socket_gbps per (backend, registered, batch, pairs) and
variant, the best of the runs (or their median with --median).
    python tools/gw_table.py DIR variant1,variant2 [--median]   (files DIR/VARIANT_R.jsonl)"""
import collections
import glob
import json
import statistics
import sys

d = collections.defaultdict(lambda: collections.defaultdict(list))
names = sys.argv[2].split(",")
for n in names:
    for f in glob.glob(f"{sys.argv[1]}/{n}_*.jsonl"):
        for line in open(f):
            if line.startswith("{"):
                x = json.loads(line)
                d[(x.get("backend", "gpu"), x["registered"], x["batch"])][(n, x["pairs"])].append(x["socket_to_socket_gbps"])
pairs = sorted({p for v in d.values() for (_, p) in v})
print("backend reg batch  " + "  ".join(f"{n:>{6 * len(pairs)}}" for n in names))
for k in sorted(d):
    cells = []
    for n in names:
        agg = statistics.median if "--median" in sys.argv else max
        cells.append("".join("%6.1f" % agg(d[k][(n, p)]) if d[k][(n, p)] else "     -" for p in pairs))
    print("%-7s %3d %5d  " % k + "  ".join(cells))
