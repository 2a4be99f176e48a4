#!/usr/bin/env python3
"""Dev tool: per-dispatch counter values of one kernel from rocprofv3 --pmc
CSV directories, in dispatch order, skipping the first `skip` dispatches
(set-up launches of the same kernel, e.g. the pre-patch pass of a VERIFY
row).  FETCH_SIZE is reported x2 (gfx950, MI355X_MICROARCH.md §HBM).

    python tools/pmc_rows.py KERNEL_SUBSTRING SKIP DIR [DIR ...]
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def rows(d, kern, skip):
    per = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(per)[skip:]
    out = {}
    for c in sorted({c for i in ids for c in per[i]}):
        v = [per[i][c] for i in ids if c in per[i]]
        m = statistics.median(v)
        if c == "FETCH_SIZE":
            out["FETCH_bytes_x2"] = round(2 * 1024 * m)
        elif c == "WRITE_SIZE":
            out["WRITE_bytes"] = round(1024 * m)
        else:
            out[c] = m
    out["dispatches"] = len(ids)
    return out


if __name__ == "__main__":
    kern, skip = sys.argv[1], int(sys.argv[2])
    for d in sys.argv[3:]:
        print(json.dumps({"dir": os.path.basename(d.rstrip("/")), **rows(d, kern, skip)}))
