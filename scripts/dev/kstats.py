#!/usr/bin/env python3
"""Dev-only: per-kernel duration summary from a rocprofv3 sqlite output (kernels view).
usage: kstats.py RESULTS.db [name-substring]"""
import sqlite3
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else "name"
rows = c.execute(f"select {name_col}, start, end from kernels order by start").fetchall()
agg = defaultdict(list)
for n, s, e in rows:
    if flt in n:
        agg[n.split("(")[0]].append((e - s) / 1e3)
for n, d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    d.sort()
    print(f"{n[:60]:60s} calls {len(d):4d} avg {sum(d)/len(d):9.1f} us  med {d[len(d)//2]:9.1f}  min {d[0]:9.1f}")
