#!/usr/bin/env python
"""Mean per-dispatch counter values per kernel from rocprofv3 counter_collection CSVs, plus
(given kernel_trace CSVs of the same runs) the mean dispatch time and the derived HBM bandwidth
FETCH_SIZE (KiB) / time and WRITE_SIZE (KiB) / time.  Usage: pmc_summary.py <csv>..."""
import collections
import csv
import sys


def main(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    meta = {}
    for p in paths:
        rows = list(csv.DictReader(open(p)))
        if not rows:
            continue
        if "Counter_Name" in rows[0]:
            for r in rows:
                k = r["Kernel_Name"]
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta[k] = (r.get("VGPR_Count"), r.get("Accum_VGPR_Count"), r.get("SGPR_Count"),
                           r.get("LDS_Block_Size"), r.get("Grid_Size"))
        elif "Start_Timestamp" in rows[0]:
            for r in rows:
                dur[r["Kernel_Name"]].append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, d in agg.items():
        print(f"{k}: vgpr/agpr/sgpr/lds/grid={meta[k]}")
        for c, v in sorted(d.items()):
            print(f"  {c:40s} {sum(v) / len(v):18.1f}  (n={len(v)})")
        t = dur.get(k)
        if t:
            # the fastest dispatches: counter collection serializes and perturbs the slow ones
            ts = sorted(t)[: max(1, len(t) // 2)]
            us = sum(ts) / len(ts)
            print(f"  {'dispatch_us (faster half, traced)':40s} {us:18.1f}  (n={len(t)})")
            for c in ("FETCH_SIZE", "WRITE_SIZE"):
                if c in d:
                    kib = sum(d[c]) / len(d[c])
                    print(f"  {c + ' GB/s':40s} {kib * 1024 / (us * 1e-6) / 1e9:18.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
