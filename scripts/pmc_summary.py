#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (scripts/pmc.sh output) per cpk:: kernel."""
import collections, csv, glob, sys
for tag in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{tag}/p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "cpk::" not in k or "generate" in k:
                continue
            kn = k.split("(")[0].replace("void ", "")
            agg[kn][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("==", tag)
    for kn, d in agg.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        wc = m.get("SQ_WAVE_CYCLES", 1)
        print(f"  {kn}: waves={m.get('SQ_WAVES',0):.0f} wave_cycles={wc:.3g} "
              f"active={m.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} wait_any={m.get('SQ_WAIT_ANY',0)/wc:.2f} "
              f"wait_inst={m.get('SQ_WAIT_INST_ANY',0)/wc:.2f}")
        print(f"     VALU={m.get('SQ_INSTS_VALU',0):.3g} SALU={m.get('SQ_INSTS_SALU',0):.3g} "
              f"LDS={m.get('SQ_INSTS_LDS',0):.3g} VMEM_RD={m.get('SQ_INSTS_VMEM_RD',0):.3g} "
              f"VMEM_WR={m.get('SQ_INSTS_VMEM_WR',0):.3g} BR={m.get('SQ_INSTS_BRANCH',0):.3g} "
              f"LDS_conflict/active={m.get('SQ_LDS_BANK_CONFLICT',0)/max(1,m.get('SQ_LDS_IDX_ACTIVE',1)):.2f} "
              f"FETCH_KB={m.get('FETCH_SIZE',0):.4g} WRITE_KB={m.get('WRITE_SIZE',0):.4g} "
              f"GRBM={m.get('GRBM_GUI_ACTIVE',0):.3g}")
