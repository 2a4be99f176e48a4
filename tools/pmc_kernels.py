#!/usr/bin/env python3
"""Dev tool: per-kernel (template-qualified name) medians of every counter in
one or more rocprofv3 --pmc CSV directories, one JSON line per kernel.
Runtime copy/fill kernels are skipped; `label` tags every line.

    python tools/pmc_kernels.py LABEL DIR [DIR ...]
"""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys


def main():
    label, dirs = sys.argv[1], sys.argv[2:]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if "rocclr" in k:
                    continue
                m = re.search(r"(k_\w+)(<[^()]*>)?", k)
                name = (m.group(1) + (m.group(2) or "")) if m else k[:60]
                per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(per.items()):
        row = {"label": label, "kernel": k, "dispatches": max(len(v) for v in cs.values())}
        row.update({c.replace("_sum", ""): statistics.median(v) for c, v in sorted(cs.items())})
        print(json.dumps(row))


if __name__ == "__main__":
    main()
