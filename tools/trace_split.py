#!/usr/bin/env python3
"""Average duration of one kernel's dispatches in a rocprofv3 kernel trace,
split by dispatch order: the first / last K dispatches of that kernel (a
bench run whose legs launch the same kernel in a known order -- e.g. the
headline's calls, then headline_rotating's).

usage: trace_split.py TRACE_DIR KERNEL_SUBSTR LAST_K [FIRST_K]  -> one JSON line
"""
import csv
import glob
import json
import os
import sys


def main():
    d, sub, last = sys.argv[1], sys.argv[2], int(sys.argv[3])
    first = int(sys.argv[4]) if len(sys.argv) > 4 else None
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    if len(rows) < last:
        sys.exit(f"{len(rows)} dispatches of {sub}, fewer than {last}")
    out = {"kernel_substr": sub, "dispatches": len(rows),
           "last": {"n": last, "avg_ns": round(sum(t for _, t in rows[-last:]) / last, 1)}}
    if first:
        out["first"] = {"n": first, "avg_ns": round(sum(t for _, t in rows[:first]) / first, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
