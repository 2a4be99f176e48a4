"""Dev tool: per-kernel summary (count, mean / min duration in us, grid) of
rocprofv3 result databases (*_results.db) under the given directories."""
import glob
import os
import sqlite3
import sys

for root in sys.argv[1:]:
    for db in sorted(glob.glob(os.path.join(root, "**", "*results.db"), recursive=True)):
        print(db)
        c = sqlite3.connect(db)
        q = ("select name, count(*), avg(duration)/1000.0, min(duration)/1000.0, grid_x from kernels "
             "group by name, grid_x order by min(start)")
        for name, cnt, avg, mn, grid in c.execute(q):
            short = name.split("(")[0].replace("icsum::(anonymous namespace)::", "")
            print(f"  {short[:60]:60s} n={cnt:4d} avg={avg:9.1f} min={mn:9.1f} grid={grid}")
