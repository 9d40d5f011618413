#!/usr/bin/env python3
"""Timeline of the batched Tunn's device work from a rocprofv3 kernel + memory-copy
trace (tools/gpu_r04_trace.sh): the device events are cut into calls at host gaps,
and per call it prints the span, the busy time per kind (input copies, AEAD
kernels, scatter kernels, small copies), their overlap, and the idle gaps.

    python tools/tunn_timeline.py DIR [--min-gap-us 500]
"""
import argparse
import csv
import glob
import json
import os


def events(d):
    ev = []
    for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            kind = ("aead" if "aead_" in name else "scatter" if "scatter" in name
                    else "blit" if "rocclr" in name else "kernel:" + name[:40])
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
    for f in glob.glob(os.path.join(d, "*memory_copy_trace.csv")):
        for r in csv.DictReader(open(f)):
            kind = "copy:" + r["Direction"].replace("MEMORY_COPY_", "").lower()
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
    ev.sort()
    return ev


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-gap-us", type=float, default=500.0)
    a = ap.parse_args()
    ev = events(a.dir)
    calls, cur, last_end = [], [], None
    for s, e, k in ev:
        if cur and s - last_end > a.min_gap_us * 1e3:
            calls.append(cur)
            cur = []
        cur.append((s, e, k))
        last_end = e if last_end is None else max(last_end, e)
    if cur:
        calls.append(cur)
    for i, c in enumerate(calls):
        t0, t1 = c[0][0], max(e for _, e, _ in c)
        kinds = sorted({k for _, _, k in c})
        busy = {k: union([(s, e) for s, e, kk in c if kk == k]) / 1e3 for k in kinds}
        count = {k: sum(1 for _, _, kk in c if kk == k) for k in kinds}
        allbusy = union([(s, e) for s, e, _ in c]) / 1e3
        print(json.dumps({"call": i, "span_us": round((t1 - t0) / 1e3, 1), "busy_any_us": round(allbusy, 1),
                          "idle_us": round((t1 - t0) / 1e3 - allbusy, 1),
                          "busy_us": {k: round(v, 1) for k, v in busy.items()}, "events": count}))


if __name__ == "__main__":
    main()
