#!/usr/bin/env python3
"""Per-launch HBM traffic of the codec kernels from scripts/gpu_bench.sh output.

FETCH_SIZE and WRITE_SIZE are in KB. On gfx950 FETCH_SIZE counts 128-B wide
streaming reads as 64 B (MI355X_MICROARCH.md §HBM), so read bytes = 2 x FETCH_SIZE
x 1024 for 16-B-per-lane streaming loads; writes are counted exactly.
Usage: pmc_traffic.py gpurun_out/TAG CONFIG_KEY [existing.json] > pmc_traffic.json
Output per config: per-kernel bytes, plus "encode" / "decode" role totals (a
decoder may be several kernels) that bench.py reports as roofline.traffic.
"""
import os
import collections
import csv
import glob
import json
import sys


def per_kernel(path, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{path}/pmc_{counter}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "cpk::" in k and r["Counter_Name"] == counter:
                vals[k.split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    path, key = sys.argv[1], sys.argv[2]
    fetch, write = per_kernel(path, "FETCH_SIZE"), per_kernel(path, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        if "generate" in k:
            continue
        rd = 2 * fetch.get(k, 0.0) * 1024
        wr = write.get(k, 0.0) * 1024
        kernels[k] = {"read_bytes": rd, "write_bytes": wr, "total_bytes": rd + wr,
                      "raw_FETCH_SIZE_KB": fetch.get(k), "raw_WRITE_SIZE_KB": write.get(k)}
    out = {"kernels": kernels}
    for role in ("encode", "decode"):
        ks = [k for k in kernels if (("encode" in k) if role == "encode" else ("decode" in k and "size" not in k))]
        if ks:
            out[role] = {"kernels": ks,
                         "read_bytes": sum(kernels[k]["read_bytes"] for k in ks),
                         "write_bytes": sum(kernels[k]["write_bytes"] for k in ks),
                         "total_bytes": sum(kernels[k]["total_bytes"] for k in ks)}
    prev = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    try:
        cur = json.load(open(prev)) if os.path.exists(prev) else {}
    except Exception:
        cur = {}
    cur[key] = out
    json.dump(cur, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
