#!/usr/bin/env python3
"""Dev-only: the last N cpk:: kernels of a rocprofv3 kernel trace as a timeline (start / end in
us from the first of them, queue id, duration). Usage: timeline.py run_kernel_trace.csv [N]"""
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "cpk::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-int(sys.argv[2] if len(sys.argv) > 2 else 40):]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cpk::", "")
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{n[:40]:40s} q{r['Queue_Id']:>3} {s:9.1f} {e:9.1f} {e - s:8.1f}")
