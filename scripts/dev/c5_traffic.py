#!/usr/bin/env python3
"""Dev-only: per-kernel HBM bytes per C5 launch from scripts/dev/pmc_c5_ab.sh output
(gpurun_out/pmc_c5_ab/NAME/{FETCH_SIZE,WRITE_SIZE}); read bytes = 2 x FETCH_SIZE KB x 1024
(gfx950 streaming-read correction, MI355X_MICROARCH.md), writes exact. Averaged per launch.
Usage: c5_traffic.py DIR [NAME ...]"""
import collections, csv, glob, os, sys

base = sys.argv[1]
for name in sys.argv[2:] or sorted(os.listdir(base)):
    tot = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = collections.defaultdict(list)
        for f in glob.glob(f"{base}/{name}/{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if "cpk::" in k and r["Counter_Name"] == c and "generate" not in k:
                    vals[k.split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
        tot[c] = {k: sum(v) / len(v) for k, v in vals.items()}
    print(f"== {name}")
    rd = wr = 0.0
    for k in sorted(set(tot["FETCH_SIZE"]) | set(tot["WRITE_SIZE"])):
        r = 2 * tot["FETCH_SIZE"].get(k, 0) * 1024 / 1e6
        w = tot["WRITE_SIZE"].get(k, 0) * 1024 / 1e6
        rd += r
        wr += w
        print(f"  {k:60s} read {r:9.1f} MB  write {w:9.1f} MB")
    print(f"  total read {rd:.1f} MB write {wr:.1f} MB (all cpk kernels of one c5 step: encode + decode)")
