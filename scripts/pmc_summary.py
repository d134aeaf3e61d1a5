#!/usr/bin/env python
"""Mean per-dispatch counter values per kernel from rocprofv3 counter_collection CSVs."""
import collections
import csv
import sys


def main(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = (r.get("VGPR_Count"), r.get("Accum_VGPR_Count"), r.get("SGPR_Count"),
                       r.get("LDS_Block_Size"), r.get("Grid_Size"))
    for k, d in agg.items():
        print(f"{k}: vgpr/agpr/sgpr/lds/grid={meta[k]}")
        for c, v in sorted(d.items()):
            print(f"  {c:40s} {sum(v) / len(v):18.1f}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1:])
