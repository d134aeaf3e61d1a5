#!/usr/bin/env python
"""Per-bin busy time of the build's device work from a gpu.sh `buildprof` run: blit copies
(D2H on this ROCm), Snappy compress / inflate, gathers, radix passes, and the SDMA copies of the
memory-copy trace, in BIN-ms bins from the first traced kernel.  Busy time sums concurrent
work, so a bin can exceed its width.

    python scripts/diag/build_timeline.py gpurun_out/X_build_ktrace.csv gpurun_out/X_build_ctrace.csv [BIN_MS]
"""
import collections
import csv
import sys


def main():
    kt, ct = sys.argv[1], sys.argv[2]
    binw = int(float(sys.argv[3]) * 1e6) if len(sys.argv) > 3 else 25 * 10 ** 6
    rows = list(csv.DictReader(open(kt)))
    cr = list(csv.DictReader(open(ct)))
    t0 = min(int(r["Start_Timestamp"]) for r in rows)
    bins = collections.defaultdict(collections.Counter)

    def add(s, e, k):
        s -= t0
        e -= t0
        b = s // binw
        while s < e:
            nb = (b + 1) * binw
            bins[b][k] += min(e, nb) - s
            s, b = nb, b + 1
    for r in rows:
        k = r["Kernel_Name"]
        k = "d2h_blit" if "copyBuffer" in k else "snappy" if "snappy_compress" in k else \
            "inflate" if "inflate" in k else "gather" if "gather" in k else \
            "radix" if "rs_" in k else "other"
        add(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k)
    for r in cr:
        add(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
            "h2d_sdma" if "HOST_TO_DEVICE" in r["Direction"] else r["Direction"].lower()[:12])
    tot = collections.Counter()
    for b in sorted(bins):
        print(f"{b * binw / 1e6:8.0f} ms  " +
              " ".join(f"{k}={v / 1e6:.0f}" for k, v in sorted(bins[b].items())))
        tot.update(bins[b])
    print("total busy ms: " + " ".join(f"{k}={v / 1e6:.0f}" for k, v in sorted(tot.items())))


if __name__ == "__main__":
    main()
