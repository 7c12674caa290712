#!/usr/bin/env python3
"""Per-kernel totals from a rocprofv3 rocpd database: python tools/prof_kernels.py run_results.db"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, count(*), sum(end - start), avg(end - start) from kernels group by name "
                 "order by sum(end - start) desc limit 40").fetchall()
for n, k, tot, avg in rows:
    print(f"{tot / 1e3:10.1f} us  {k:6d} x {avg / 1e3:8.2f} us  {n[:110]}")
