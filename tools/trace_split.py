"""Split a rocprofv3 kernel trace's dispatches by what the GPU was doing when
each one started, and report per-kernel duration medians per class:

  back_to_back  the previous dispatch (any queue) ended at most GAP_US before
  idle_queue    nothing ran for more than GAP_US before it started
  overlapped    it started while another dispatch was still running

A kernel-stats average mixes the three (a single call starts
from an idle queue, a back-to-back one does not, and two streams overlap).
usage: python tools/trace_split.py run_kernel_trace.csv[.gz] [KERNEL_SUBSTR ...] [--gap-us 2]
(profiles/r5_stack_kernel_trace_min.csv.gz: the round-5 stack rows' trace,
names trimmed to the kernel template, timestamps as recorded ->
profiles/r5_stack_trace_split.jsonl)"""
import argparse
import csv
import gzip
import json
import re
import statistics


def load(path):
    rows = []
    with (gzip.open(path, "rt") if path.endswith(".gz") else open(path)) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def classify(rows, gap_ns):
    out = []
    busy_until = None
    for s, e, name in rows:
        if busy_until is None or s - busy_until > gap_ns:
            cls = "idle_queue"
        elif s < busy_until:
            cls = "overlapped"
        else:
            cls = "back_to_back"
        out.append((name, cls, (e - s) / 1e3))
        busy_until = e if busy_until is None else max(busy_until, e)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("kernels", nargs="*", help="substrings of the kernel names to report (default: every kernel)")
    ap.add_argument("--gap-us", type=float, default=2.0)
    a = ap.parse_args()
    per = {}
    for name, cls, us in classify(load(a.trace), a.gap_us * 1e3):
        if a.kernels and not any(k in name for k in a.kernels):
            continue
        per.setdefault(name, {}).setdefault(cls, []).append(us)
    for name, d in sorted(per.items()):
        m = re.search(r"(k_\w+<[^>]*>|k_\w+)", name)
        row = {"kernel": m.group(1) if m else name[:120], "gap_us": a.gap_us}
        for cls in ("back_to_back", "idle_queue", "overlapped"):
            v = d.get(cls, [])
            row[cls] = {"dispatches": len(v), "median_us": round(statistics.median(v), 2) if v else None,
                        "min_us": round(min(v), 2) if v else None}
        print(json.dumps(row))


if __name__ == "__main__":
    main()
