#!/usr/bin/env python3
"""Dev-only: per-kernel read/write MB (FETCH_SIZE x 2, WRITE_SIZE; MI355X_MICROARCH §HBM and
scripts/dev/fetch_calib.hip) and the C5 leg times from scripts/dev/c5_fetch_ab.sh output."""
import collections, csv, glob, json, os, sys
out = sys.argv[1]
for d in sorted(glob.glob(f"{out}/*/")):
    vals = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        acc = collections.defaultdict(list)
        for f in glob.glob(f"{d}pmc_{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                if "cpk::" in k and "generate" not in k:
                    acc[k].append(float(r["Counter_Value"]))
        vals[c] = {k: sum(v) / len(v) for k, v in acc.items()}
    print("==", os.path.basename(d.rstrip("/")))
    for k in sorted(set(vals["FETCH_SIZE"]) | set(vals["WRITE_SIZE"])):
        rd = 2 * vals["FETCH_SIZE"].get(k, 0) * 1024 / 1e6
        wr = vals["WRITE_SIZE"].get(k, 0) * 1024 / 1e6
        if rd + wr > 1:
            print(f"  {k[:48]:48s} read {rd:8.1f} MB  write {wr:8.1f} MB")
legs = f"{out}/legs.log"
if os.path.exists(legs):
    cur = None
    for line in open(legs):
        if line.startswith("=="):
            cur = line.split()[1]
        elif line.strip():
            c5 = json.loads(line)["c5"]
            print(f"{cur:30s} encode {c5['encode_ms']:.4f} ms  decode {c5['decode_ms']:.4f} ms")
