#!/usr/bin/env python3
"""Dev: per-call kernel timeline of a rocprofv3 kernel trace (calls split at class_count_kernel)."""
import csv, sys
r = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x['Start_Timestamp']))
nm = lambda x: x['Kernel_Name'].split('(')[0].replace('void ', '')
groups, cur = [], None
for x in r:
    if nm(x).startswith('cpk::class_count_kernel'):
        cur = [x]; groups.append(cur)
    elif cur is not None:
        cur.append(x)
for g in groups[-2:]:
    t0 = int(g[0]['Start_Timestamp'])
    print('----')
    for x in g[:14]:
        if not nm(x).startswith('cpk::'):
            continue
        s, e = int(x['Start_Timestamp']) - t0, int(x['End_Timestamp']) - t0
        print(f"  {nm(x)[:44]:44s} {s/1e3:8.1f} .. {e/1e3:8.1f}  ({(e-s)/1e3:7.1f} us)")
