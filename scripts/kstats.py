#!/usr/bin/env python3
"""Print name / calls / average µs of each kernel in rocprofv3 *_kernel_stats.csv files."""
import csv, sys
for f in sys.argv[1:]:
    print("==", f)
    for r in csv.DictReader(open(f)):
        name = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]
        print(f"  {name:60s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.1f} min_us={float(r['MinNs'])/1e3:9.1f}")
