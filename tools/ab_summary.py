#!/usr/bin/env python3
"""Dev tool: median per (row, build) of interleaved A/B rows (tools/probe/ab_libs.sh
output).  Usage: python tools/ab_summary.py FILE.jsonl [key=us]"""
import collections
import json
import statistics
import sys

key = sys.argv[2] if len(sys.argv) > 2 else "us"
acc = collections.defaultdict(list)
order = []
for line in open(sys.argv[1]):
    d = json.loads(line)
    row = d.get("config") or d.get("row")
    if row not in order:
        order.append(row)
    if key in d:
        acc[(row, d.get("lib", "-"))].append(d[key])
libs = sorted({k[1] for k in acc}, key=lambda x: [k[1] for k in acc].index(x))
print("row".ljust(40), *[x[:18].rjust(18) for x in libs])
for row in order:
    print(row[:40].ljust(40), *[(f"{statistics.median(acc[(row, l)]):.2f}" if acc.get((row, l)) else "-").rjust(18)
                                  for l in libs])
