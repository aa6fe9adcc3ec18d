#!/usr/bin/env python3
"""Top kernels of a rocprofv3 sqlite output (rocpd): kstats_db.py RUN.db [N] -> name, calls, avg ms, total ms"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
rows = c.execute(f"select {name}, count(*), avg(end - start), sum(end - start) from kernels group by {name} "
                 "order by sum(end - start) desc").fetchall()
for nm, cnt, avg, tot in rows[:n]:
    print(f"{tot / 1e6:9.2f} ms {cnt:5d} {avg / 1e6:8.3f}  {str(nm)[:110]}")
